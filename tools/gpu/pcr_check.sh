#!/bin/bash
# GPU box: the -m gpu suite + bench on the in-tree library, then paired comparisons against an
# experiment variant (config 2 bench rounds, and the config 4 / 5 likelihood benches).
#   bash tools/gpu/pcr_check.sh TAG VARIANT
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VAR=$2
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu/run_tests_bench.sh $TAG || exit 1
timeout -k 10 600 python tools/ab_bench.py 4 $VAR base > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 2; }
tail -2 $O/ab.jsonl
for r in 1 2 3; do
for c in config4 config5; do
  for v in $VAR base; do
    L=$PWD/emri_frequencydomainwaveforms_amd/libemrifd.so
    [ $v != base ] && L=$PWD/exp/libemrifd_$v.so
    EFD_LIB=$L timeout -k 10 200 python bench.py --likelihood $c --api-steps 0 > $O/like_${c}_$v.json 2> $O/like_${c}_$v.err || { tail -5 $O/like_${c}_$v.err; exit 3; }
    python -c "import json;d=json.load(open('$O/like_${c}_$v.json'));print('$c','$v',round(d['value']),round(d['ms_per_step'],3))"
  done
done
done
