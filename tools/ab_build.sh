#!/bin/bash
# A/B variants of the ICP kernel: tools/ab_build.sh NAME "-DFLAG=1 ..." -> ab/NAME/libslamhip.so
# (select with SLAMHIP_LIB=ab/NAME/libslamhip.so; ab/ is git-ignored)
set -e
cd "$(dirname "$0")/../icp-slam-with-loop-closure_amd/csrc"
make -s
OUT=../../ab/$1
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
    -I../../include $2 -c icp_kernels.hip -o $OUT/icp_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libslamhip.so $OUT/icp_kernels.o \
    build/pgo_kernels.o build/gn_kernels.o build/gn_bcr.o build/grid_kernels.o
echo built $OUT/libslamhip.so
