#!/bin/bash
# GPU box, round 6: config 5's fused groups rotating over 2 streams (default) against 4, and
# groups of 8 over 4 streams: rotated configs.py rounds and the host timers of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
for i in 1 2 3; do
NAME=d2; run python tools/configs.py --only 5 --reps 9 --no-cpu-baseline
NAME=d4; EFD_FUSED_DEPTH=4 run python tools/configs.py --only 5 --reps 9 --no-cpu-baseline
NAME=g8d4; EFD_FUSED_DEPTH=4 EFD_FUSED_GROUP=8 run python tools/configs.py --only 5 --reps 9 --no-cpu-baseline
NAME=hs_d2; run python tools/halfstep_host.py config5
NAME=hs_d4; EFD_FUSED_DEPTH=4 run python tools/halfstep_host.py config5
NAME=hs_g8d4; EFD_FUSED_DEPTH=4 EFD_FUSED_GROUP=8 run python tools/halfstep_host.py config5
done
echo dp done
