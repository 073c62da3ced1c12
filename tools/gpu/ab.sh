#!/bin/bash
# GPU box: paired A/B of library variants through bench.py (tools/ab_bench.py), optionally after
# a subset of the GPU tests.   bash tools/gpu/ab.sh TAG ROUNDS "VARIANTS" ["PYTEST -k EXPR"]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ROUNDS=$2; VARIANTS=$3; TESTK=$4
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$TESTK" > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python tools/ab_bench.py $ROUNDS $VARIANTS > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
grep SUMMARY $O/ab.jsonl
