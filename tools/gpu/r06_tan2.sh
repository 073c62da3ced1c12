#!/bin/bash
# GPU box, round 6: the envelope records' sin/cos in the tangent form with the amplitude prescaled by COS_A and -r^2/2 in one product (in-tree; the
# tangent form of r06_tan.sh, exp/libemrifd_tan1.so)
# : the full -m gpu suite on the new kernel, then paired headline rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/ab_bench.py 5 tan1 base > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
grep SUMMARY $O/ab.jsonl
echo tan2 done
