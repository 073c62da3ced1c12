#!/bin/bash
# GPU box, round 6: paired A/B (optional) and the API half-step traces of configs 5 and 4.
#   bash tools/gpu/r06_api.sh TAG ROUNDS "VARIANTS"
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ROUNDS=$2; VARIANTS=$3
O=gpurun_out/$TAG; mkdir -p $O
if [ "$ROUNDS" != "0" ]; then
  timeout -k 10 900 python tools/ab_bench.py $ROUNDS $VARIANTS > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
  grep SUMMARY $O/ab.jsonl
fi
for c in config5 config4; do
  timeout -k 10 300 python tools/api_trace.py $c 6 > $O/api_$c.jsonl 2> $O/api_$c.err || { tail -20 $O/api_$c.err; exit 6; }
  tail -2 $O/api_$c.jsonl
done
