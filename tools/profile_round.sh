#!/bin/bash
# Collect the round's GPU evidence on an MI355X box (run through gpurun from the repo root):
#   gpu parity tests, one bench line (with CPU baseline), the rocprofv3 kernel-trace summary of
#   the same bench command, and separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters) for
#   k_modesum. Raw output goes to gpurun_out/<tag>/; tools/summarize_profiles.py turns it into
#   the committed files under profiles/.
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
cat $O/bench.json
timeout -k 10 300 python tools/td_vs_fd.py > $O/td_vs_fd.json 2> $O/td_vs_fd.err || { tail -20 $O/td_vs_fd.err; exit 8; }
cat $O/td_vs_fd.json
cd /tmp && export TMPDIR=/tmp
# the same command as the bench line (overlap pipeline): one k_modesum launch per waveform on
# the sum stream, so the profiled per-launch durations are the quantity the bench reports
B="$R/bench.py --no-cpu-baseline --steps 50 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $B > $O/trace.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_modesum --output-format csv -d $O/pmc_fetch -o run -- python $B > $O/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_modesum --output-format csv -d $O/pmc_write -o run -- python $B > $O/pmc_write.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_modesum --output-format csv -d $O/pmc_sq -o run -- python $B > $O/pmc_sq.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-include-regex k_modesum --output-format csv -d $O/pmc_valu -o run -- python $B > $O/pmc_valu.log 2>&1 || exit 7
echo done
