#!/bin/bash
# A/B of the fused-frames accumulation: on the main stream vs overlapped on its own stream
# (RT_ACCUM_OVERLAP), with the main build and a register-capped variant (RT_ACCUM_VGPRS=32).
# usage: scripts/ab_overlap.sh [extra bench args...]
set -u
mkdir -p gpurun_out
one() {  # one <label> [env...]
  local label=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 "${EXTRA[@]}") || exit $?
  echo "$label $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["ms_per_frame"], r["kernel_ms"], r.get("accum_ms_per_launch"))')"
}
EXTRA=("$@")
V=mini-opencl-raytracer_amd/lib/variants/librt_hip_v32.so
for rep in 1 2; do
  one main_ov0 RT_ACCUM_OVERLAP=0
  one main_ov1 RT_ACCUM_OVERLAP=1
  one v32_ov0 RT_ACCUM_OVERLAP=0 RT_HIP_LIB=$V
  one v32_ov1 RT_ACCUM_OVERLAP=1 RT_HIP_LIB=$V
done | tee -a gpurun_out/ab_overlap.txt
