#!/bin/bash
# GPU box: the HIP = host-twin fold comparison (tests/test_gpu_twin.py, config 3's grid) with
# experiment libraries in place of the product (EFD_LIB), parity records per variant.
#   bash tools/gpu/twin_study.sh TAG VARIANT...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
for v in "$@"; do
  O=gpurun_out/$TAG/twin_$v; mkdir -p $O
  LIB=exp/libemrifd_$v.so; [ "$v" = base ] && LIB=emri_frequencydomainwaveforms_amd/libemrifd.so
  EFD_LIB=$PWD/$LIB EFD_PARITY_OUT=$PWD/$O timeout -k 10 400 python -u -m pytest tests/test_gpu_twin.py tests/test_gpu_configs.py -k "twin" -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?
  tail -2 $O/pytest.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
