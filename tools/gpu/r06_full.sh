#!/bin/bash
# GPU box, round 6: full -m gpu suite (parity records), paired A/B, host scaling, chain trace.
#   bash tools/gpu/r06_full.sh TAG ROUNDS "VARIANTS"
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ROUNDS=$2; VARIANTS=$3
O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
if [ "$ROUNDS" != "0" ]; then
  timeout -k 10 900 python tools/ab_bench.py $ROUNDS $VARIANTS > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
  grep SUMMARY $O/ab.jsonl
fi
timeout -k 10 300 python tools/host_scaling.py > $O/host_scaling.json 2>&1 || exit 6
cat $O/host_scaling.json
bash tools/gpu/chain_trace.sh $TAG || exit 7
exit $rc
