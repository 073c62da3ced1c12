#!/bin/bash
# GPU box: configs 4 and 5 (tools/configs.py) under library / environment variants, rotated
# ROUNDS times, then the kernel timeline of the in-tree build (tools/gpu/chain_trace.sh).
#   bash tools/gpu/chain_ab.sh TAG ROUNDS "NAME:LIB:ENV" ...   (LIB "-" = in-tree, ENV "-" = none)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ROUNDS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    IFS=: read name lib envs <<< "$spec"
    L=$PWD/emri_frequencydomainwaveforms_amd/libemrifd.so
    [ "$lib" != "-" ] && L=$PWD/$lib
    E=(); [ "$envs" != "-" ] && E=(${envs//,/ })
    env EFD_LIB=$L "${E[@]}" timeout -k 10 300 python tools/configs.py --only 4,5 --reps 3 > $O/cfg_${name}_$r.jsonl 2> $O/cfg_${name}_$r.err || { tail -20 $O/cfg_${name}_$r.err; exit 2; }
    python -c "
import json,sys
for l in open('$O/cfg_${name}_$r.jsonl'):
    d=json.loads(l); print('$name', $r, d['config'][:8], round(d['device_loglikes_per_s']), round(d['api_loglikes_per_s']))
"
  done
done
bash tools/gpu/chain_trace.sh $TAG
