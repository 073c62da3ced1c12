#!/bin/bash
# GPU box, round 6: configs 4/5 API rates with each walker's mode selection on one OpenMP thread
# (EFD_PREFETCH_SPLIT=0) against the pool's share per walker (default): rotated rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
for i in 1 2 3; do
NAME=split1; run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
NAME=split0; EFD_PREFETCH_SPLIT=0 run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
done
echo ps done
