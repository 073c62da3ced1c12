#!/bin/bash
# GPU box: the batch / likelihood GPU tests, then interleaved config 4 / 5 likelihood benches
# with and without the fused sum's empty-tile constants (efd_loglike_tile_constants).
#   bash tools/gpu/tilec_check.sh TAG [ROUNDS]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; R=${2:-3}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch_prepare.py tests/test_gpu_api.py tests/test_gpu_pe_configs.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in $(seq $R); do
for c in config4 config5; do
  for v in on off; do
    F=""; [ $v = off ] && F="--no-tile-constants"
    timeout -k 10 200 python bench.py --likelihood $c --api-steps 0 $F > $O/like_${c}_$v.json 2> $O/like_${c}_$v.err || { tail -5 $O/like_${c}_$v.err; exit 3; }
    python -c "import json;d=json.load(open('$O/like_${c}_$v.json'));print('$c','$v',round(d['value']),round(d['ms_per_step'],3))" | tee -a $O/rounds.txt
  done
done
done
