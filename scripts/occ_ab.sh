#!/bin/bash
set -u
for rep in 1 2; do
for lib in librt_hip.so librt_hip_p5.so; do for m in pinned devicelib; do
  out=$(RT_HIP_LIB=$PWD/mini-opencl-raytracer_amd/lib/$lib timeout -k 10 120 python bench.py --math $m --no-cpu-baseline --steps 4 --warmup 1) || exit $?
  echo "$lib $m $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')"
done; done; done | tee gpurun_out/occ_ab.txt
