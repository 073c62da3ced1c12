#!/bin/bash
# GPU box, round 6 closing run on the final tree (the kernels unchanged since r06zz's PMC pass):
# the full -m gpu suite (parity records), the bench line, configs 1/3/4/5 with their CPU
# baselines, and config 4/5 half-step timers.   bash tools/gpu/r06_close.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
cat $O/bench.json
timeout -k 10 600 python tools/configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 3; }
for c in config4 config5; do
  timeout -k 10 200 python tools/halfstep_host.py $c > $O/hs_$c.json 2>> $O/hs.err || exit 4
done
echo close done
