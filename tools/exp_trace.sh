#!/bin/bash
# Kernel-trace stats of experiment variants (run through gpurun from the repo root):
#   bash tools/exp_trace.sh OUTTAG VARIANT...
# one rocprofv3 --kernel-trace --stats run of tools/exp_variants.py's child per variant; prints
# each kernel's call count and mean duration.
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/$v \
    -o run -- python $R/tools/exp_variants.py child $v > $R/gpurun_out/$TAG/$v.log 2>&1 || exit 1
  echo "== $v"
  python - "$R/gpurun_out/$TAG/$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:70]:70s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
