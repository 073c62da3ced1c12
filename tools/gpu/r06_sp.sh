#!/bin/bash
# GPU box, round 6: the envelope fit made before k_items' grid-bound loads (speculative) against
# after them: twin/modesum tests, paired headline rounds, config-4/5 chain traces of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_twin.py tests/test_gpu_modesum.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 7; }
timeout -k 10 700 python tools/ab_bench.py 3 nospec base > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
grep SUMMARY $O/ab.jsonl
export TMPDIR=/tmp
for v in base nospec; do
  L=$PWD/emri_frequencydomainwaveforms_amd/libemrifd.so; [ $v = nospec ] && L=$PWD/exp/libemrifd_nospec.so
  EFD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr4_$v -o run -- python bench.py --likelihood config4 --steps 20 --warmup 2 --api-steps 0 > $O/tr4_$v.log 2>&1 || exit 6
done
echo sp done
