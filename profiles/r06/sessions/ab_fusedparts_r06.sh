#!/bin/bash
# Round 6 experiment: fused launches of multi-GPU ranks (<= 16 M work items) with the small-launch hand-out
# (no bulk region, static first chunks, 8 partitioned tail counters; variant fp) -- fused parity tests on
# fp under a rank-sized launch, then the emulated N = 8 fused ranks at tail chunks 256 / 128 / 64.
set -u
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_fp.so timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py tests/test_comm.py tests/test_benched_path.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fp_tests.txt 2>&1 || { tail -30 gpurun_out/fp_tests.txt; exit 1; }
tail -1 gpurun_out/fp_tests.txt
O=gpurun_out/fp_emu.txt; : > $O
for rep in 1 2; do
 for l in main fp; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_fp.so; fi
  for t in 256 128 64; do
   for sc in cornell bunny; do
    RT_EMU_TUNE="tail_chunk=$t" RT_EMU_FUSED=1 RT_EMU_SCENE=$sc RT_EMU_STEPS=10 timeout -k 10 300 python scripts/rank_emulation.py 8 > gpurun_out/fp_last.txt 2>&1 || exit 1
    echo "$l $sc tail$t N=8 $(grep -o 'max [0-9.]*' gpurun_out/fp_last.txt)" | tee -a $O
   done
  done
 done
done
