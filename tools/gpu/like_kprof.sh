#!/bin/bash
# GPU box: kernel-trace statistics of the config 4 / 5 likelihood benches for the in-tree library
# and experiment variants.   bash tools/gpu/like_kprof.sh TAG VARIANT[,VARIANT2...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VARS=${2//,/ }
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for c in config4 config5; do
  for v in base $VARS; do
    L=$PWD/emri_frequencydomainwaveforms_amd/libemrifd.so
    [ $v != base ] && L=$PWD/exp/libemrifd_$v.so
    EFD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${c}_$v -o run -- python bench.py --likelihood $c --steps 20 --warmup 2 --api-steps 0 > $O/prof_${c}_$v.log 2>&1 || { tail -20 $O/prof_${c}_$v.log; exit 2; }
    python - $O/prof_${c}_$v/run_kernel_stats.csv $c $v <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in r:
    n = x['Name']
    if any(k in n for k in ('k_modesum_batch', 'k_ll_final', 'k_prep_pcr_b', 'k_items')):
        print(sys.argv[2], sys.argv[3], n.split('(')[0][-40:], x['Calls'], round(float(x['AverageNs']) / 1e3, 1), 'us')
PY
  done
done
