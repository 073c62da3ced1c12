#!/bin/bash
# GPU box, round 6: the API rate's run-to-run swing (configs 4/5 in one process, alone, with
# passive OpenMP waiting) and the half-step trace in tools/configs.py's order.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
NAME=c45; run python tools/configs.py --only 4,5 --reps 5 --no-cpu-baseline
NAME=c45; run python tools/configs.py --only 4,5 --reps 5 --no-cpu-baseline
NAME=c5; run python tools/configs.py --only 5 --reps 5 --no-cpu-baseline
NAME=c45passive; OMP_WAIT_POLICY=PASSIVE run python tools/configs.py --only 4,5 --reps 5 --no-cpu-baseline
NAME=c45passive; OMP_WAIT_POLICY=PASSIVE run python tools/configs.py --only 4,5 --reps 5 --no-cpu-baseline
NAME=trace45; run python tools/api_trace.py config4,config5 6
echo api2 done
