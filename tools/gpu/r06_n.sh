#!/bin/bash
# GPU box, round 6: where the walker chains and the config-5 half-step go now (kernel/copy
# traces, host section timers), and the headline's per-kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
bash tools/gpu/chain_trace.sh $TAG || exit 5
for c in config4 config5; do
  timeout -k 10 200 python tools/halfstep_host.py $c > $O/hs_$c.json 2> $O/hs_$c.err || { tail -20 $O/hs_$c.err; exit 6; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/head -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 3 > $GRAFT_REPO_ROOT/$O/head.log 2>&1 || exit 7
echo n done
