#!/bin/bash
# GPU box, round 6: envelope fit by fixed matrices (parity + headline), then the API rate's
# run-to-run swing (configs 4/5 in one process, alone, with passive OpenMP waiting).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_twin.py tests/test_gpu_modesum.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 7; }
NAME=head; run python bench.py --steps 20 --warmup 3
NAME=head; run python bench.py --steps 20 --warmup 3
NAME=c45; run python tools/configs.py --only 4,5 --reps 5 --no-cpu-baseline
NAME=c45; run python tools/configs.py --only 4,5 --reps 5 --no-cpu-baseline
NAME=c5; run python tools/configs.py --only 5 --reps 5 --no-cpu-baseline
NAME=c45passive; OMP_WAIT_POLICY=PASSIVE run python tools/configs.py --only 4,5 --reps 5 --no-cpu-baseline
NAME=trace45; run python tools/api_trace.py config4,config5 6
echo api3 done
