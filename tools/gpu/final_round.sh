#!/bin/bash
# GPU box: the round's closing measurements at HEAD. Full -m gpu suite (parity records to
# $O/parity), then tools/gpu/pmc_refresh.sh (bench line, kernel trace, PMC passes), then
# tools/configs.py (configs 1, 3, 4, 5 and test.sh's windowed one) and the walker half-step
# host phases of configs 4 and 5.   bash tools/gpu/final_round.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu/pmc_refresh.sh $TAG || exit $?
timeout -k 10 600 python tools/configs.py --only 1,3,4,5,w --reps 5 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 8; }
timeout -k 10 200 python tools/halfstep_host.py config4 > $O/halfstep4.json 2>&1 || exit 9
timeout -k 10 200 python tools/halfstep_host.py config5 > $O/halfstep5.json 2>&1 || exit 10
echo final done
