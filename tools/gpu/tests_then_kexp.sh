#!/bin/bash
# GPU box: selected -m gpu tests (parity records to $O/parity), then tools/gpu/kexp.sh. A test
# failure (rc 1) still runs the experiments; any other failure (timeout, abort, fault) stops.
#   bash tools/gpu/tests_then_kexp.sh TAG "TESTS" ROUNDS base NAME...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; TESTS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export EFD_PARITY_OUT=$PWD/$O/parity
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu/kexp.sh $TAG "$@"
