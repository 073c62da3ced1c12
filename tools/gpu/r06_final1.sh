#!/bin/bash
# GPU box, round 6 closing measurements, part 1: the full -m gpu suite (parity records), then
# the bench line + kernel trace + PMC passes (pmc_refresh.sh).   bash tools/gpu/r06_final1.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/pmc_refresh.sh $TAG || exit $?
echo final1 done
