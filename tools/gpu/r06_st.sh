#!/bin/bash
# GPU box, round 6: config 4/5 staging copy on 16 OpenMP threads (exp/libemrifd_st16.so) against
# 8 (in-tree): rotated configs.py rounds and the config-5 host timers of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pe_configs.py tests/test_gpu_api.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 7; }
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
for i in 1 2 3; do
NAME=st8; run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
NAME=st16; EFD_LIB=$PWD/exp/libemrifd_st16.so run python tools/configs.py --only 4,5 --reps 9 --no-cpu-baseline
done
timeout -k 10 200 python tools/halfstep_host.py config5 > $O/hs8.json 2> $O/hs8.err || exit 9
EFD_LIB=$PWD/exp/libemrifd_st16.so timeout -k 10 200 python tools/halfstep_host.py config5 > $O/hs16.json 2> $O/hs16.err || exit 10
echo st done
