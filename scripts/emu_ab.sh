set -u
for rep in 1 2; do
for l in main old; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  RT_EMU_FUSED=1 timeout -k 10 200 python scripts/rank_emulation.py 1 8 > gpurun_out/emu_$l.log 2>&1 || exit 1
  echo "$l $(grep '^N=8' gpurun_out/emu_$l.log | sed 's/.*| max/max/') | $(grep '^N=1' gpurun_out/emu_$l.log | sed 's/.*| max/max/')"
done
done
unset RT_HIP_LIB
