#!/bin/bash
# GPU box, round 6: preparation kernels capped at 64 VGPRs (two of their waves in one of the sum's
# 128-VGPR slots) against uncapped: paired headline rounds, GPU twin/modesum tests, chain trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_twin.py tests/test_gpu_modesum.py tests/test_gpu_pe_configs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 7; }
timeout -k 10 900 python tools/ab_bench.py 3 nopack base > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
grep SUMMARY $O/ab.jsonl
bash tools/gpu/chain_trace.sh $TAG || exit 6
echo s done
