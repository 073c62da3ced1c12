#!/bin/bash
# GPU box: interleaved A/B of bench.py --likelihood CONFIG over variants, R rounds. A variant is
# a space-separated list of NAME=VALUE environment settings and --bench-args ("-" = neither).
#   bash tools/gpu/like_ab2.sh TAG CONFIG ROUNDS variant...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; C=$2; R=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    envs=(); args=()
    for tok in $v; do
      case $tok in -) ;; --*) args+=("$tok") ;; *) envs+=("$tok") ;; esac
    done
    env "${envs[@]}" timeout -k 10 200 python bench.py --likelihood $C --steps 40 --warmup 4 --api-steps 0 "${args[@]}" > $O/ab_${C}_r${r}_v$i.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 3; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']))" $O/ab_${C}_r${r}_v$i.json "$v" $C
    i=$((i+1))
  done
done
