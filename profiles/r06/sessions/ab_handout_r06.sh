#!/bin/bash
# Round 6: the new work hand-out defaults (static first tail chunk, per-frame counter slots,
# per-workgroup tail share) against the old ones (lib/variants/librt_hip_old.so): the GPU suite on the
# new build, then bench configurations and emulated N = 8 ranks, interleaved.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/handout_suite.txt 2>&1 || { tail -30 gpurun_out/handout_suite.txt; exit 1; }
tail -1 gpurun_out/handout_suite.txt
O=gpurun_out/handout_ab.txt; : > $O
V=mini-opencl-raytracer_amd/lib/variants/librt_hip_old.so
for rep in 1 2 3; do
  for l in main old; do
    if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V; fi
    for cfg in "c2|--width 1920 --height 1080 --bounces 2 --frames 1 --steps 40" "c2t512|--width 1920 --height 1080 --bounces 2 --frames 1 --steps 40 --tune tail_chunk=512" "cornell|" "bunny|--scene bunny" "pf4k|--launch per-frame"; do
      n=${cfg%%|*}; args=${cfg#*|}
      timeout -k 10 120 python bench.py --no-cpu-baseline --no-configs --no-drop-in --steps 10 $args > gpurun_out/ho_last.json 2>&1 || exit 1
      python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/ho_last.json') if l.startswith('{')][-1])
print('$l', '$n', 'ms/frame', d['ms_per_frame'], 'launch_ms', d['roofline'].get('launch_ms'))" | tee -a $O
    done
  done
done
for l in main old; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V; fi
  for f in 1 0; do
    RT_EMU_FUSED=$f RT_EMU_SCENE=cornell RT_EMU_STEPS=10 timeout -k 10 300 python scripts/rank_emulation.py 1 8 > gpurun_out/ho_emu.txt 2>&1 || exit 1
    echo "== $l fused=$f" | tee -a $O; grep "N=" gpurun_out/ho_emu.txt | tee -a $O
  done
done
unset RT_HIP_LIB
