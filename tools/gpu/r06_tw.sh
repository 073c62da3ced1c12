#!/bin/bash
# GPU box, round 6 experiment: the windowed rows kernel with its twiddle powers left out
# (exp/libemrifd_notw.so: wrong transforms, timing only: the bound a cheaper twiddle could reach)
# against the in-tree kernel, kernel traces of the windowed half-steps on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="$R/tools/windowed_profile.py 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o run -- python $P > $O/base.log 2>&1 || exit 3
EFD_LIB=$R/exp/libemrifd_notw.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/notw -o run -- python $P > $O/notw.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base2 -o run -- python $P > $O/base2.log 2>&1 || exit 5
echo tw done
