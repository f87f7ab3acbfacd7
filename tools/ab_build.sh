#!/bin/bash
# A/B variants of the library: tools/ab_build.sh NAME "-DFLAG=1 ..." -> ab/NAME/libslamhip.so
# (every source rebuilt with the flags; select with SLAMHIP_LIB=ab/NAME/libslamhip.so; ab/ is git-ignored)
# -DSLAM_TIMING_ONLY is added: the ablation switches (SLAM_ABL_*, ...) refuse to compile without it
set -e
cd "$(dirname "$0")/../icp-slam-with-loop-closure_amd/csrc"
OUT=../../ab/$1
mkdir -p $OUT
objs=""
for f in icp_kernels pgo_kernels gn_kernels gn_bcr gn_bcr_gj grid_kernels; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
      -I../../include -DSLAM_TIMING_ONLY $2 -c $f.hip -o $OUT/$f.o &
  objs="$objs $OUT/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libslamhip.so $objs
echo built $OUT/libslamhip.so
