#!/bin/bash
# GPU box: likelihood-path GPU tests, tools/configs.py (configs 1, 3, 4, 5), bench.py
# --likelihood for configs 4 and 5 (device + API rates), host overhead per walker.
#   bash tools/gpu/final_like.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 500 python -u -m pytest tests/test_gpu_batch_prepare.py tests/test_gpu_api.py tests/test_gpu_pe_configs.py tests/test_gpu_parallel.py tests/test_gpu_likelihood.py -m gpu -v --timeout 300 --timeout-method thread > $O/like_tests.log 2>&1 || { tail -30 $O/like_tests.log; exit 1; }
tail -2 $O/like_tests.log
timeout -k 10 500 python tools/configs.py --reps 5 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 2; }
for c in config4 config5; do
  timeout -k 10 300 python bench.py --likelihood $c --steps 40 --warmup 4 --api-steps 4 > $O/like_$c.json 2> $O/like_$c.err || { tail -20 $O/like_$c.err; exit 3; }
  cat $O/like_$c.json
done
for c in 4 5; do
  timeout -k 10 300 python tools/host_overhead.py --config $c --reps 3 > $O/host_c$c.txt 2>&1 || { tail -20 $O/host_c$c.txt; exit 4; }
  grep wall_ms $O/host_c$c.txt
done
