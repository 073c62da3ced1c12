#!/bin/bash
# GPU box: rocprofv3 kernel-trace summary of tools/configs.py --only ONLY (one pass).
#   bash tools/gpu/profile_configs.sh TAG ONLY [configs args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; ONLY=$2; shift 2
O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/tools/configs.py --only $ONLY "$@" > $O/configs.jsonl 2> $O/trace.log || { tail -20 $O/trace.log; exit 3; }
cat $O/configs.jsonl | head -c 600
echo
head -25 $O/trace/run_kernel_stats.csv
