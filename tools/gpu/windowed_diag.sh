#!/bin/bash
# GPU box: SQ counter passes (LDS, wait and VALU cycles) of the windowed likelihood's FFT and
# reduction kernels, one pass each.   bash tools/gpu/windowed_diag.sh TAG [ENV=VALUE ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
P="$R/tools/windowed_profile.py 3"
K='k_fc_|k_hann_loglike'
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-include-regex "$K" --output-format csv -d $O/diag1 -o run -- python $P > $O/diag1.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F SQ_THREAD_CYCLES_VALU --kernel-include-regex "$K" --output-format csv -d $O/diag2 -o run -- python $P > $O/diag2.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d $O/diag3 -o run -- python $P > $O/diag3.log 2>&1 || exit 5
cd $R && python tools/windowed_diag.py $TAG
