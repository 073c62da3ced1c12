#!/bin/bash
# GPU box, round 6: paired A/B, chain trace, configs 4/5 three times (API spread).
#   bash tools/gpu/r06_probe.sh TAG ROUNDS "VARIANTS"
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ROUNDS=$2; VARIANTS=$3
O=gpurun_out/$TAG; mkdir -p $O
if [ "$ROUNDS" != "0" ]; then
  timeout -k 10 900 python tools/ab_bench.py $ROUNDS $VARIANTS > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
  grep SUMMARY $O/ab.jsonl
fi
bash tools/gpu/chain_trace.sh $TAG || exit 7
for i in 1 2 3; do
  timeout -k 10 300 python tools/configs.py --only 4,5 --reps 5 --no-cpu-baseline >> $O/configs45.jsonl 2>> $O/configs45.err || { tail -20 $O/configs45.err; exit 8; }
done
echo probe done
