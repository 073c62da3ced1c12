#!/bin/bash
# GPU box, round 6: the windowed logL reduced inside the inverse column pass
# (efd_hann_loglike_local): parity, paired rates against the mirror-pair form, the GC probe,
# then the windowed kernel trace + HBM PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_windowed.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 7; }
run() { timeout -k 10 300 "$@" >> $O/$NAME.jsonl 2>> $O/$NAME.err || { tail -20 $O/$NAME.err; exit 8; }; }
for i in 1 2; do
NAME=w_local; run python tools/configs.py --only w --reps 5 --no-cpu-baseline
NAME=w_pair; run python tools/configs.py --only w --reps 5 --no-cpu-baseline --hann-pair
done
NAME=gc5; run python tools/gc_cycles.py config5
bash tools/gpu/windowed_prof.sh $TAG
echo win done
