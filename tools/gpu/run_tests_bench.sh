#!/bin/bash
# GPU box: the -m gpu suite (parity records to $O/parity) then one bench line.
#   bash tools/gpu/run_tests_bench.sh TAG [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}; shift
O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error:|assert " $O/pytest.log | head -30; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
cat $O/bench.json
