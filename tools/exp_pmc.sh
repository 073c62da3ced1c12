#!/bin/bash
# PMC pass over k_modesum for experiment variants (run through gpurun from the repo root):
#   bash tools/exp_pmc.sh OUTTAG VARIANT...
# one rocprofv3 --pmc run per variant; CSVs under gpurun_out/<OUTTAG>/<variant>/
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
PMC=${EXP_PMC:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}
for v in "$@"; do
  timeout -k 10 200 rocprofv3 --pmc $PMC --kernel-include-regex k_modesum --output-format csv \
    -d $R/gpurun_out/$TAG/$v -o run -- python $R/tools/exp_variants.py child $v > $R/gpurun_out/$TAG/$v.log 2>&1 || exit 1
done
python $R/tools/exp_pmc_summary.py $R/gpurun_out/$TAG "$@"
