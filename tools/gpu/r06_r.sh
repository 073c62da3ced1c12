#!/bin/bash
# GPU box, round 6: the staged fused inverse (parity, profile, paired rates), then the headline's
# preparation kernels alone under a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu/r06_q.sh $TAG || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prep -o run -- python $GRAFT_REPO_ROOT/tools/prep_only.py 20 > $GRAFT_REPO_ROOT/$O/prep.log 2>&1 || exit 9
echo r done
