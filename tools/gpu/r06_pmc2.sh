#!/bin/bash
# GPU box, round 6: bench line, kernel trace and PMC passes on the final kernel source (after the
# tangent-form envelope sin/cos), plus config 4/5 chain traces.   bash tools/gpu/r06_pmc2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
bash tools/gpu/pmc_refresh.sh $TAG || exit $?
echo pmc2 done
