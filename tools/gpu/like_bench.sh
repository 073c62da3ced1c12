#!/bin/bash
# GPU box: the sharded-likelihood GPU test, then bench.py --likelihood for configs 4 and 5.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parallel.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_parallel.log 2>&1 || { tail -30 $O/pytest_parallel.log; exit 1; }
tail -2 $O/pytest_parallel.log
for c in config4 config5; do
  timeout -k 10 300 python bench.py --likelihood $c --steps 20 --warmup 4 > $O/like_$c.json 2> $O/like_$c.err || { tail -20 $O/like_$c.err; exit 2; }
  cat $O/like_$c.json
done
