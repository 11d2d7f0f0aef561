#!/bin/bash
# Round 6: counter partitions as the default (main: 8 partitions, per-wave tail rule) against p1 (one
# counter, per-workgroup rule) -- the GPU suite on main, then config 2, 512^2 per-frame and 4K per-frame,
# and the emulated N = 8 per-frame rank.
set -u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/parts2_suite.txt 2>&1 || { tail -30 gpurun_out/parts2_suite.txt; exit 1; }
tail -1 gpurun_out/parts2_suite.txt
O=gpurun_out/parts2_ab.txt; : > $O
for r in 1 2; do
 for l in main p1; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  for cfg in "c2|--width 1920 --height 1080 --bounces 2 --frames 1 --steps 40" "c512pf|--width 512 --height 512 --bounces 9 --frames 8 --launch per-frame" "pf4k|--launch per-frame"; do
   n=${cfg%%|*}; args=${cfg#*|}
   timeout -k 10 120 python bench.py --no-cpu-baseline --no-configs --no-drop-in --steps 10 $args > gpurun_out/parts2_last.json 2>&1 || exit 1
   python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/parts2_last.json') if l.startswith('{')][-1])
print('$l', '$n', 'ms/frame', d['ms_per_frame'], 'launch_ms', d['roofline'].get('launch_ms'))" | tee -a $O
  done
 done
done
for l in main p1; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  RT_EMU_FUSED=0 RT_EMU_SCENE=cornell RT_EMU_STEPS=5 timeout -k 10 300 python scripts/rank_emulation.py 8 > gpurun_out/parts2_emu.txt 2>&1 || exit 1
  echo "$l per-frame N=8 $(grep -o 'max [0-9.]*' gpurun_out/parts2_emu.txt)" | tee -a $O
done
