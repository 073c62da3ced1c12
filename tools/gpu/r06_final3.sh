#!/bin/bash
# GPU box, round 6 closing run on the final source: the full -m gpu suite (parity records), a
# paired headline A/B of k_items' grid (K-sized, items1, against the final), then the bench line,
# kernel trace and PMC passes (pmc_refresh.sh).   bash tools/gpu/r06_final3.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/ab_bench.py 3 items1 base > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
grep SUMMARY $O/ab.jsonl
bash tools/gpu/pmc_refresh.sh $TAG || exit $?
echo final3 done
