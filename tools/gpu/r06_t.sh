#!/bin/bash
# GPU box, round 6: one native call per fused group (efd_fused_group): the pe-config parity tests,
# then configs 4/5 rotated rounds native / Python groups, and the config-5 host timers.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pe_configs.py tests/test_gpu_api.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 7; }
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
for i in 1 2 3; do
NAME=native; run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
NAME=pygroups; run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline --python-groups
done
timeout -k 10 200 python tools/halfstep_host.py config5 > $O/hs5.json 2> $O/hs5.err || exit 9
timeout -k 10 200 python tools/halfstep_host.py config5 python > $O/hs5py.json 2> $O/hs5py.err || exit 10
echo t done
