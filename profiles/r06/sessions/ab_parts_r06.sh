#!/bin/bash
# Round 6 experiment: tail counters split over partitions (RT_COUNTER_PARTS, variants p4 / p8) for per-frame
# launches without a bulk region -- per-frame parity tests on p8, then config 2 at tail chunks 256 / 128 / 64.
set -u
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_p8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_interactive.py tests/test_benched_path.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parts_tests.txt 2>&1 || { tail -30 gpurun_out/parts_tests.txt; exit 1; }
tail -1 gpurun_out/parts_tests.txt
O=gpurun_out/parts_ab.txt; : > $O
for r in 1 2 3; do
 for l in main p4 p8; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  for t in 256 128 64; do
   timeout -k 10 120 python bench.py --no-cpu-baseline --no-configs --no-drop-in --width 1920 --height 1080 --bounces 2 --frames 1 --steps 40 --tune tail_chunk=$t > gpurun_out/parts_last.json 2>&1 || exit 1
   python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/parts_last.json') if l.startswith('{')][-1])
print('$l', 'c2 tail$t', 'ms/frame', d['ms_per_frame'], 'launch_ms', d['roofline'].get('launch_ms'))" | tee -a $O
  done
 done
done
