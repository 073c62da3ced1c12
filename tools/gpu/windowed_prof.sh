#!/bin/bash
# GPU box: the windowed likelihood's kernel trace (timed region cut by markers) and the HBM PMC
# passes of its row/column/reduction kernels.   bash tools/gpu/windowed_prof.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 300 python tools/windowed_profile.py 5 > $O/windowed.json 2> $O/windowed.err || { tail -20 $O/windowed.err; exit 2; }
cat $O/windowed.json
cd /tmp && export TMPDIR=/tmp
P="$R/tools/windowed_profile.py 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wtrace -o run -- python $P > $O/wtrace.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_fc_|k_hann_|k_modesum' --output-format csv -d $O/wpmc_fetch -o run -- python $P > $O/wpmc_fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_fc_|k_hann_|k_modesum' --output-format csv -d $O/wpmc_write -o run -- python $P > $O/wpmc_write.log 2>&1 || exit 5
echo windowed prof done
