#!/bin/bash
# GPU box: interleaved A/B of tools/configs.py --only ONLY under environment variants.
#   bash tools/gpu/configs_ab.sh TAG ONLY ROUNDS variant...   ("-" = no extra environment)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ONLY=$2; R=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    env $( [ "$v" = "-" ] || echo $v ) timeout -k 10 300 python tools/configs.py --only $ONLY --reps 5 > $O/cab_r${r}_v$i.jsonl 2> $O/cab.err || { tail -20 $O/cab.err; exit 3; }
    python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['config'][:8], round(d.get('device_waveforms_per_s', d.get('device_loglikes_per_s', 0))))" $O/cab_r${r}_v$i.jsonl "$v"
    i=$((i+1))
  done
done
