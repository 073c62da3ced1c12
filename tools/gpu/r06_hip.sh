#!/bin/bash
# GPU box, round 6: HIP API trace of config 5's half-steps (the per-group launch costs).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=$PWD/gpurun_out/$TAG; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d $O/hip -o run -- python $R/tools/halfstep_host.py config5 > $O/hip.log 2>&1 || exit 3
echo hip done
