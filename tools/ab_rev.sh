#!/bin/bash
# Build the library of a git revision into ab/NAME (A/B against the working tree):
#   tools/ab_rev.sh NAME [REV=HEAD]
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=${2:-HEAD}
TMP=$(mktemp -d)
for f in icp_kernels pgo_kernels gn_kernels gn_bcr gn_bcr_gj grid_kernels common gn_bcr; do
  ext=hip; [ $f = common ] && ext=hpp; [ $f = gn_bcr ] && git -C "$REPO" show $REV:icp-slam-with-loop-closure_amd/csrc/gn_bcr.hpp > $TMP/gn_bcr.hpp
  git -C "$REPO" show $REV:icp-slam-with-loop-closure_amd/csrc/$f.$ext > $TMP/$f.$ext
done
git -C "$REPO" show $REV:include/slamhip.h > $TMP/slamhip.h
mkdir -p "$REPO/ab/$NAME"
for f in icp_kernels pgo_kernels gn_kernels gn_bcr gn_bcr_gj grid_kernels; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$TMP -c $TMP/$f.hip -o $TMP/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$REPO/ab/$NAME/libslamhip.so" $TMP/*.o
rm -rf $TMP
echo built ab/$NAME from $REV
