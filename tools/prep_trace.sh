#!/bin/bash
# usage: prep_trace.sh OUTDIR VARIANT...
O=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/emri_frequencydomainwaveforms_amd/libemrifd.so; else L=$R/exp/libemrifd_$v.so; fi
  EFD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$O/$v -o run -- python3 $R/tools/td_vs_fd.py > $R/gpurun_out/$O/$v.log 2>&1 || exit 1
done
