#!/bin/bash
# GPU box, round 6: config 4/5 half-step host timers (three runs each) and the fused-likelihood
# tests, after the per-group host path's caching (workspace floor, template, data pointers).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pe_configs.py tests/test_gpu_api.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 7; }
for i in 1 2 3; do
  for c in config5 config4; do
    timeout -k 10 200 python tools/halfstep_host.py $c >> $O/hs_$c.jsonl 2>> $O/hs.err || exit 9
    timeout -k 10 200 python tools/halfstep_host.py $c python >> $O/hspy_$c.jsonl 2>> $O/hs.err || exit 10
  done
done
echo hs done
