#!/bin/bash
# GPU box, round 6: the envelope records. Full -m gpu suite (parity records to $O/parity), then
# paired A/B of the headline with and without envelope records (EFD_ENV=0).
#   bash tools/gpu/r06_env.sh TAG [ROUNDS]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ROUNDS=${2:-3}
O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python tools/ab_bench.py $ROUNDS base base@env:EFD_ENV=0 > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
grep SUMMARY $O/ab.jsonl
exit $rc
