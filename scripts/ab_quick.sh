#!/bin/bash
# Interleaved A/B of library variants (mini-opencl-raytracer_amd/lib/variants/librt_hip_*.so) vs the
# main build on the default bench: ms/frame and KernelEntry ms per launch, REPS rounds.
# usage: scripts/ab_quick.sh REPS [bench args...]
set -u
mkdir -p gpurun_out
reps=$1; shift
V=mini-opencl-raytracer_amd/lib/variants
for rep in $(seq $reps); do
  for l in main $(ls $V 2>/dev/null | sed -n 's/^librt_hip_\(.*\)\.so$/\1/p'); do
    if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V/librt_hip_$l.so; fi
    timeout -k 10 100 python bench.py --no-cpu-baseline --steps 10 "$@" > gpurun_out/abq_$l.json || exit 1
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/abq_$l.json') if l.startswith('{')][-1])
print('$l', d['ms_per_frame'], d['roofline'].get('launch_ms', d['roofline'].get('kernel_ms')))" | tee -a gpurun_out/ab_quick.txt
  done
done
