#!/bin/bash
# GPU box: host-side profile (tools/host_overhead.py) and a rocprofv3 kernel trace of the
# likelihood bench for configs 4 and 5.   bash tools/gpu/like_profile.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for c in 4 5; do
  timeout -k 10 300 python tools/host_overhead.py --config $c --reps 3 > $O/host_c$c.txt 2>&1 || { tail -20 $O/host_c$c.txt; exit 1; }
  tail -3 $O/host_c$c.txt
done
for c in config4 config5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python bench.py --likelihood $c --steps 6 --warmup 2 --api-steps 0 > $O/prof_$c.log 2>&1 || { tail -20 $O/prof_$c.log; exit 2; }
done
find $O -name "*kernel_stats.csv" | head
