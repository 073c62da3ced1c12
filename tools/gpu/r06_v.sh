#!/bin/bash
# GPU box, round 6: k_items with a smaller grid at large K (threads take several records):
# parity tests, then paired headline rounds against the K-sized grid (items1) and a quarter more.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_modesum.py tests/test_gpu_twin.py tests/test_gpu_batch_prepare.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 7; }
timeout -k 10 900 python tools/ab_bench.py 3 ${VARIANTS:-items1 base items8} > $O/ab.jsonl 2>&1 || { tail -5 $O/ab.jsonl; exit 5; }
grep SUMMARY $O/ab.jsonl
echo v done
