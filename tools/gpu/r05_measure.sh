#!/bin/bash
# GPU box, round 5.   bash tools/gpu/r05_measure.sh TAG PART
#   PART pmc:     the bench line + kernel trace + PMC passes (pmc_refresh.sh) and an LDS pass of
#                 the mode sum
#   PART configs (configs_only: without the windowed passes): the windowed path's trace and HBM passes, configs 1/3/4/5 (API and device
#                 rates), the API path's upstream overlap A/B (EFD_PREFETCH_ASYNC, EFD_FUSED_GROUP),
#                 the walker half-step host phases and the upstream pool's scaling
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; PART=$2; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
if [ "$PART" = pmc ]; then
  bash tools/gpu/pmc_refresh.sh $TAG || exit $?
  cd /tmp && export TMPDIR=/tmp
  B="$R/bench.py --no-cpu-baseline --steps 50 --warmup 5"
  timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-include-regex k_modesum --output-format csv -d $O/pmc_lds -o run -- python $B > $O/pmc_lds.log 2>&1 || { tail -5 $O/pmc_lds.log; exit 8; }
  echo pmc done
  exit 0
fi
[ "$PART" = configs_only ] || bash tools/gpu/windowed_prof.sh $TAG || exit $?
timeout -k 10 600 python tools/configs.py --only 1,3,4,5 --reps 5 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 9; }
timeout -k 10 300 env EFD_PREFETCH_ASYNC=0 python tools/configs.py --only 4,5 --reps 5 > $O/configs_sync.jsonl 2> $O/configs_sync.err || { tail -20 $O/configs_sync.err; exit 9; }
timeout -k 10 300 env EFD_FUSED_GROUP=4 python tools/configs.py --only 4 --reps 5 > $O/configs_g4.jsonl 2> $O/configs_g4.err || { tail -20 $O/configs_g4.err; exit 9; }
timeout -k 10 200 python tools/halfstep_host.py config4 > $O/halfstep4.json 2>&1 || exit 10
timeout -k 10 200 python tools/halfstep_host.py config5 > $O/halfstep5.json 2>&1 || exit 11
timeout -k 10 200 python tools/upstream_scaling.py 8 > $O/upstream8.json 2>&1 || exit 12
echo measure done
