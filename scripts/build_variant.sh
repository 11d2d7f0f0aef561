#!/bin/bash
# Build an experimental librt_hip.so with extra compile flags, for A/B runs on the GPU box:
#   scripts/build_variant.sh NAME "-DRT_STEP_BURST=2 ..."  ->  mini-opencl-raytracer_amd/lib/variants/librt_hip_NAME.so
# Select it at run time with RT_HIP_LIB=<path> (clrt/_native.py).
set -eu
NAME=$1; FLAGS=${2:-}
HERE=$(cd "$(dirname "$0")/../mini-opencl-raytracer_amd" && pwd)
OUT=$HERE/lib/variants; OBJ=$HERE/build/variants/$NAME
mkdir -p $OUT $OBJ
F="--offload-arch=gfx950 -O2 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize $FLAGS"
/opt/rocm/bin/hipcc $F -c $HERE/csrc/rt_kernels.hip -o $OBJ/rt_kernels.o &
/opt/rocm/bin/hipcc $F -fno-hip-fp32-correctly-rounded-divide-sqrt -c $HERE/csrc/rt_kernels_shipped.hip -o $OBJ/rt_kernels_shipped.o &
/opt/rocm/bin/hipcc $F -c $HERE/csrc/rt_capi.cpp -o $OBJ/rt_capi.o &
/opt/rocm/bin/hipcc $F -Wno-unused-result -c $HERE/csrc/rt_bvh.hip -o $OBJ/rt_bvh.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/librt_hip_$NAME.so $OBJ/rt_kernels.o $OBJ/rt_kernels_shipped.o $OBJ/rt_capi.o $OBJ/rt_bvh.o
echo $OUT/librt_hip_$NAME.so
