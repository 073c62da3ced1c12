#!/bin/bash
# GPU box: the batch / likelihood / edge GPU tests on the in-tree library, then interleaved
# config 4 / 5 likelihood benches of the in-tree library ("base") against an experiment variant
# (exp/libemrifd_VARIANT.so).   bash tools/gpu/like_ab.sh TAG VARIANT[,VARIANT2...] [ROUNDS]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VARS=${2//,/ }; R=${3:-3}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch_prepare.py tests/test_gpu_api.py tests/test_gpu_pe_configs.py \
  tests/test_gpu_edges.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in $(seq $R); do
for c in config4 config5; do
  for v in base $VARS; do
    L=$PWD/emri_frequencydomainwaveforms_amd/libemrifd.so
    [ $v != base ] && L=$PWD/exp/libemrifd_$v.so
    EFD_LIB=$L timeout -k 10 200 python bench.py --likelihood $c --api-steps 0 > $O/like_${c}_$v.json 2> $O/like_${c}_$v.err || { tail -5 $O/like_${c}_$v.err; exit 3; }
    python -c "import json;d=json.load(open('$O/like_${c}_$v.json'));print('$c','$v',round(d['value']),round(d['ms_per_step'],3))" | tee -a $O/rounds.txt
  done
done
done
