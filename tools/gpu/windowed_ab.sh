#!/bin/bash
# GPU box: the windowed tests, then ROUNDS rotated windowed half-step timings (tools/
# windowed_profile.py) under environment variants, then the windowed trace/PMC passes.
#   bash tools/gpu/windowed_ab.sh TAG ROUNDS VARIANT...   ("-" = no extra environment)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_windowed.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_w.log 2>&1
rc=$?; tail -2 $O/pytest_w.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest_w.log | head -20; exit 1; }
for r in $(seq 1 $R); do
  for v in "$@"; do
    env $( [ "$v" = "-" ] || echo $v ) timeout -k 10 300 python tools/windowed_profile.py 5 > $O/wab.json 2> $O/wab.err || { tail -5 $O/wab.err; exit 2; }
    python -c "
import json,sys
d=json.load(open(sys.argv[1])); print('WAB', sys.argv[2], sys.argv[3], round(d['ms_per_half_step'],3), d.get('ll_sha16'))" $O/wab.json "$v" $r
  done
done
bash tools/gpu/windowed_prof.sh $TAG
