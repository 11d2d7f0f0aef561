#!/bin/bash
# Round 6: work-hand-out variants (static first chunk, per-frame counter slots, per-workgroup tail
# share) -- parity tests on the combined variant, then every variant against main (ab_session.sh).
set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_all3.so timeout -k 10 600 python -u -m pytest tests/test_benched_path.py tests/test_gpu_parity.py tests/test_fused_frames.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_sched_tests.txt 2>&1 || { tail -30 gpurun_out/ab_sched_tests.txt; exit 1; }
tail -1 gpurun_out/ab_sched_tests.txt
AB_CONFIGS="c2 --width 1920 --height 1080 --bounces 2 --frames 1 --steps 40;cornell;bunny --scene bunny;pf4k --launch per-frame" bash scripts/ab_session.sh 3
