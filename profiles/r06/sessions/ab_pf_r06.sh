#!/bin/bash
# Round 6: per-frame ring fill loading the stored value ahead of the root visit (main) vs after it
# (lib/variants/librt_hip_late.so): per-frame parity tests, then config 2, 4K per-frame, 512^2 per-frame.
set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_interactive.py tests/test_benched_path.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pf_tests.txt 2>&1 || { tail -30 gpurun_out/pf_tests.txt; exit 1; }
tail -1 gpurun_out/pf_tests.txt
for r in 1 2 3; do
 for l in main late; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_late.so; fi
  for cfg in "c2|--width 1920 --height 1080 --bounces 2 --frames 1 --steps 40" "pf4k|--launch per-frame" "c512pf|--width 512 --height 512 --bounces 9 --frames 8 --launch per-frame"; do
   n=${cfg%%|*}; args=${cfg#*|}
   timeout -k 10 120 python bench.py --no-cpu-baseline --no-configs --no-drop-in --steps 10 $args > gpurun_out/pf_last.json 2>&1 || exit 1
   python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/pf_last.json') if l.startswith('{')][-1])
print('$l', '$n', 'ms/frame', d['ms_per_frame'], 'launch_ms', d['roofline'].get('launch_ms'))"
  done
 done
done
