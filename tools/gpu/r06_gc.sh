#!/bin/bash
# GPU box, round 6: the API half-step's stalls -- garbage collections per call (gc callbacks),
# with and without gc.freeze() after setup.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
NAME=trace; run python tools/api_trace.py config4,config5 12
NAME=freeze; TRACE_GC_FREEZE=1 run python tools/api_trace.py config4,config5 12
echo gc done
