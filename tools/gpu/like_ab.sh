#!/bin/bash
# GPU box: likelihood-path tests, host profile, then bench.py --likelihood for configs 4 and 5
# under environment variants ("NAME=VALUE ..." strings, "-" for none).
#   bash tools/gpu/like_ab.sh TAG [variant ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch_prepare.py tests/test_gpu_api.py tests/test_gpu_pe_configs.py tests/test_gpu_parallel.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/quick.log 2>&1 || { tail -30 $O/quick.log; exit 1; }
tail -2 $O/quick.log
for c in 4 5; do
  timeout -k 10 300 python tools/host_overhead.py --config $c --reps 3 > $O/host_c$c.txt 2>&1 || { tail -20 $O/host_c$c.txt; exit 2; }
  grep wall_ms $O/host_c$c.txt
done
i=0
for v in "${@:--}"; do
  for c in config4 config5; do
    env $( [ "$v" = "-" ] || echo $v ) timeout -k 10 300 python bench.py --likelihood $c --steps 20 --warmup 4 > $O/like_${c}_v$i.json 2> $O/like_${c}_v$i.err || { tail -20 $O/like_${c}_v$i.err; exit 3; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']), round(d['api_loglikes_per_s']))" $O/like_${c}_v$i.json "$v" $c
  done
  i=$((i+1))
done
