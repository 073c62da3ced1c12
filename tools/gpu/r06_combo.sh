#!/bin/bash
# GPU box, round 6: parity subset, a paired A/B, then r06_measure.sh.
#   bash tools/gpu/r06_combo.sh TAG ROUNDS "VARIANTS" "PYTEST -k EXPR" [MEASURE PARTS]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ROUNDS=$2; VARIANTS=$3; TESTK=$4; PARTS=${5:-pmc,like,scan,c1}
O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$TESTK" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
if [ "$ROUNDS" != "0" ]; then
  timeout -k 10 900 python tools/ab_bench.py $ROUNDS $VARIANTS > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
  grep SUMMARY $O/ab.jsonl
fi
bash tools/gpu/r06_measure.sh $TAG $PARTS
