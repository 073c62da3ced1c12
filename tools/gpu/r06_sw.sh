#!/bin/bash
# GPU box, round 6: the sparse fused sum's workgroup count (EFD_SPARSE_WG) and split threshold
# (EFD_SPLIT_MIN_COST) on configs 4 and 5: rotated configs.py rounds, device rates.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
for i in 1 2 3; do
NAME=base; run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
NAME=wg2048; EFD_SPARSE_WG=2048 run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
NAME=wg8192; EFD_SPARSE_WG=8192 run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
NAME=sc24; EFD_SPLIT_MIN_COST=24 run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
NAME=sc96; EFD_SPLIT_MIN_COST=96 run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
done
echo sw done
