#!/bin/bash
# Render speed of the host SAH tree vs the device-built linear BVH (rtBuildBVH).
set -u
mkdir -p gpurun_out
for sc in cornell bunny; do for b in host device; do
  timeout -k 10 200 python bench.py --scene $sc --bvh $b --no-cpu-baseline --steps 3 > gpurun_out/bvh_${sc}_$b.log 2>&1 || exit $?
  echo "$sc $b $(grep ms_per gpurun_out/bvh_${sc}_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"], d["config"]["rays_per_step"])')" | tee -a gpurun_out/bvh_ab.txt
done; done
