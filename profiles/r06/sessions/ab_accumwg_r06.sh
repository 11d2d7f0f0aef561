#!/bin/bash
# Round 6: accumulation workgroups of 1 / 2 waves (variants aw1, aw2) against main -- 4K fused Cornell and
# the emulated N = 8 fused rank (the accumulation gates the render two launches later: the N = 8 chain).
set -u
AB_CONFIGS="cornell" bash scripts/ab_session.sh 2 || exit 1
O=gpurun_out/aw_emu.txt; : > $O
for rep in 1 2; do
 for l in main aw1 aw2; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  RT_EMU_FUSED=1 RT_EMU_SCENE=cornell RT_EMU_STEPS=10 timeout -k 10 300 python scripts/rank_emulation.py 8 > gpurun_out/aw_last.txt 2>&1 || exit 1
  echo "$l cornell N=8 $(grep -o 'max [0-9.]*' gpurun_out/aw_last.txt)" | tee -a $O
 done
done
