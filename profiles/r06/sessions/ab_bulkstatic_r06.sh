#!/bin/bash
# Round 6 experiment: static first chunks in the bulk region (RT_STATIC_FIRST_BULK; sfb16: only launches of
# <= 16 M work items, i.e. N = 8 ranks) against main -- benched-path parity on sfb, 4K fused Cornell / bunny,
# and the emulated N = 8 fused ranks.
set -u
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_sfb.so timeout -k 10 600 python -u -m pytest tests/test_benched_path.py tests/test_fused_frames.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sfb_tests.txt 2>&1 || { tail -30 gpurun_out/sfb_tests.txt; exit 1; }
tail -1 gpurun_out/sfb_tests.txt
AB_CONFIGS="cornell;bunny --scene bunny" bash scripts/ab_session.sh 2 || exit 1
O=gpurun_out/sfb_emu.txt; : > $O
for rep in 1 2; do
 for l in main sfb sfb16; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  for sc in cornell bunny; do
   RT_EMU_FUSED=1 RT_EMU_SCENE=$sc RT_EMU_STEPS=10 timeout -k 10 300 python scripts/rank_emulation.py 8 > gpurun_out/sfb_last.txt 2>&1 || exit 1
   echo "$l $sc N=8 $(grep -o 'max [0-9.]*' gpurun_out/sfb_last.txt)" | tee -a $O
  done
 done
done
