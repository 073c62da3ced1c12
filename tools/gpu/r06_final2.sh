#!/bin/bash
# GPU box, round 6 closing measurements, part 2: tools/configs.py (configs 1, 3, 4, 5, windowed),
# the likelihood and scan bench lines with their CPU baselines, the windowed profile, chain traces
# and half-step host timers.   bash tools/gpu/r06_final2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python tools/configs.py --only 1,3,4,5,w --reps 7 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 8; }
bash tools/gpu/r06_measure.sh $TAG like,scan || exit 9
bash tools/gpu/windowed_prof.sh $TAG || exit 10
bash tools/gpu/chain_trace.sh $TAG || exit 11
for c in config4 config5; do
  timeout -k 10 200 python tools/halfstep_host.py $c > $O/halfstep_$c.json 2> $O/halfstep_$c.err || exit 12
done
echo final2 done
