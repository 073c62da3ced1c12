#!/bin/bash
# GPU box: kernel variants (exp/libemrifd_<NAME>.so, tools/exp_variants.py build): one
# exp_variants run (k_modesum ms on config 2, the spectrum's max deviation from the in-tree
# library's), then ROUNDS paired rounds of bench.py through tools/ab_bench.py.
#   bash tools/gpu/kexp.sh TAG ROUNDS base NAME...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python tools/exp_variants.py run "$@" > $O/variants.jsonl 2> $O/variants.err || { tail -20 $O/variants.err; exit 3; }
cat $O/variants.jsonl
[ "$R" -gt 0 ] || exit 0
timeout -k 10 900 python tools/ab_bench.py $R "$@" > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 4; }
grep SUMMARY $O/ab.jsonl
