#!/bin/bash
# GPU box: one bench line, the rocprofv3 kernel-trace summary of the same command, and the PMC
# passes tools/summarize_profiles.py turns into profiles/<TAG>_* and profiles/pmc_traffic.json.
#   bash tools/gpu/pmc_refresh.sh TAG [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --steps 50 --warmup 5 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $B > $O/trace.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_modesum --output-format csv -d $O/pmc_fetch -o run -- python $B > $O/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_modesum --output-format csv -d $O/pmc_write -o run -- python $B > $O/pmc_write.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex k_modesum --output-format csv -d $O/pmc_sq -o run -- python $B > $O/pmc_sq.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --kernel-include-regex k_modesum --output-format csv -d $O/pmc_valu -o run -- python $B > $O/pmc_valu.log 2>&1 || exit 7
echo pmc done
