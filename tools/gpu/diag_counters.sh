#!/bin/bash
# GPU box: the counters rocprofv3 offers here, and stall / LDS counters of k_modesum_batch over
# the bench command (one PMC pass per block budget).
#   bash tools/gpu/diag_counters.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
B="$R/bench.py --no-cpu-baseline --steps 20 --warmup 5 $*"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-include-regex k_modesum --output-format csv -d $O/pmc_lds -o run -- python $B > $O/pmc_lds.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex k_modesum --output-format csv -d $O/pmc_sq2 -o run -- python $B > $O/pmc_sq2.log 2>&1 || exit 5
echo diag done
