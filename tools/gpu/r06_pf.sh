#!/bin/bash
# GPU box, round 6: the fused windowed pass with the epilogue data (dl, wl) double-buffered 4 deep, the first 4 requested before the transform,
# against 8 deep after it (exp/libemrifd_base.so): parity, paired
# windowed half-steps, the windowed profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_windowed.py -k "local or test_sh" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 7; }
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
for i in 1 2; do
NAME=pf; run python tools/configs.py --only w --reps 7 --no-cpu-baseline
NAME=base; EFD_LIB=$PWD/exp/libemrifd_base.so run python tools/configs.py --only w --reps 7 --no-cpu-baseline
done
bash tools/gpu/windowed_prof.sh $TAG || exit 6
echo pf done
