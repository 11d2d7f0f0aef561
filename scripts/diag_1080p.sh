#!/bin/bash
# Diagnostic session for BASELINE config 2 (1080p, 2 bounces, one per-frame launch): the wave timeline
# (RT_TIMELINE build, 5-us bins), the per-phase profile (stats build) and a kernel trace of bench.py.
set -o pipefail
mkdir -p gpurun_out/t1080
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_tl8.so RT_TL_W=1920 RT_TL_H=1080 RT_TL_LB=2 RT_TL_FRAMES=1 RT_TL_DIV=8 timeout -k 10 180 python scripts/timeline.py 1 > gpurun_out/t1080/timeline.txt 2>&1 &&
RT_PHASE_W=1920 RT_PHASE_H=1080 RT_PHASE_MATH=shipped RT_PHASE_LB=2 RT_PHASE_FRAMES=1 timeout -k 10 180 python scripts/phase_profile.py > gpurun_out/t1080/phase.txt 2>&1 &&
export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t1080/prof -o run -- python3 bench.py --width 1920 --height 1080 --bounces 2 --frames 1 --steps 20 --warmup 3 --no-configs --no-cpu-baseline --no-drop-in > gpurun_out/t1080/bench.txt 2>&1
