#!/bin/bash
# Build an experimental librt_hip.so with extra compile flags, for A/B runs on the GPU box:
#   scripts/build_variant.sh NAME "-DRT_NODE_BURST=4 ..."  ->  mini-opencl-raytracer_amd/lib/variants/librt_hip_NAME.so
# (the product Makefile with its own object/library directories).  Select it at run time with
# RT_HIP_LIB=<path> (clrt/_native.py); scripts/ab_quick.sh runs every variant against the main build.
set -eu
NAME=$1; FLAGS=${2:-}
HERE=$(cd "$(dirname "$0")/../mini-opencl-raytracer_amd" && pwd)
OBJ=$HERE/build/variants/$NAME
mkdir -p $HERE/lib/variants $OBJ
make -s -C $HERE OBJDIR=$OBJ LIBDIR=$OBJ EXTRA_HIPFLAGS="$FLAGS" $OBJ/librt_hip.so
cp $OBJ/librt_hip.so $HERE/lib/variants/librt_hip_$NAME.so
echo $HERE/lib/variants/librt_hip_$NAME.so
