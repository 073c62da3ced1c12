#!/bin/bash
# GPU box: the -m gpu suite, one bench line, config 3's scan line, then a paired A/B of library
# variants (tools/ab_bench.py).   bash tools/gpu/tests_bench_ab.sh TAG ROUNDS VARIANT...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ROUNDS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu/run_tests_bench.sh $TAG || exit $?
timeout -k 10 300 python bench.py --scan config3 --steps 5 --warmup 1 > $O/scan.json 2> $O/scan.err || { tail -20 $O/scan.err; exit 3; }
cat $O/scan.json
timeout -k 10 1200 python tools/ab_bench.py $ROUNDS "$@" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 4; }
grep SUMMARY $O/ab.jsonl
