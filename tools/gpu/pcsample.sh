#!/bin/bash
# GPU box: rocprofv3 PC sampling (beta) of k_modesum over a short bench run.
#   bash tools/gpu/pcsample.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --kernel-include-regex k_modesum --output-format csv -d $O/pcs -o run -- python $R/bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/pcs.log 2>&1; rc=$?
tail -5 $O/pcs.log; ls -la $O/pcs 2>/dev/null | head
exit 0
