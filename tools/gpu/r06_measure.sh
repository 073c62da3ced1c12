#!/bin/bash
# GPU box, round 6: the headline line + kernel trace + PMC passes (pmc_refresh.sh), then the
# likelihood, scan and config-1 lines with their host-twin CPU baselines.
#   bash tools/gpu/r06_measure.sh TAG [PARTS: any of pmc,like,scan,c1]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; PARTS=${2:-pmc,like,scan,c1}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
if [[ $PARTS == *pmc* ]]; then
  bash tools/gpu/pmc_refresh.sh $TAG || exit $?
fi
if [[ $PARTS == *like* ]]; then
  timeout -k 10 300 python bench.py --likelihood config4 --steps 20 --warmup 3 > $O/like4.json 2> $O/like4.err || { tail -20 $O/like4.err; exit 11; }
  timeout -k 10 300 python bench.py --likelihood config5 --steps 20 --warmup 3 > $O/like5.json 2> $O/like5.err || { tail -20 $O/like5.err; exit 12; }
fi
if [[ $PARTS == *scan* ]]; then
  timeout -k 10 300 python bench.py --scan config3 --steps 3 --warmup 1 > $O/scan3.json 2> $O/scan3.err || { tail -20 $O/scan3.err; exit 13; }
fi
if [[ $PARTS == *c1* ]]; then
  timeout -k 10 300 python tools/configs.py --only 1 --reps 5 > $O/config1.jsonl 2> $O/config1.err || { tail -20 $O/config1.err; exit 14; }
fi
echo measure done
