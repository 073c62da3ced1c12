#!/bin/bash
# GPU box: kernel and copy timeline of the config 4 / 5 fused-likelihood half-steps (for
# tools/chain_timeline.py).   bash tools/gpu/chain_trace.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for c in config4 config5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_$c -o run -- python bench.py --likelihood $c --steps 20 --warmup 2 --api-steps 0 > $O/tr_$c.log 2>&1 || { tail -20 $O/tr_$c.log; exit 2; }
done
