# fused rank emulation (N = 1 and 8) of the main build and every lib/variants library, interleaved
set -u
mkdir -p gpurun_out
V=mini-opencl-raytracer_amd/lib/variants
out=gpurun_out/emu_variants.txt; rm -f $out
for rep in 1 2; do
for l in main $(ls $V 2>/dev/null | sed -n 's/^librt_hip_\(.*\)\.so$/\1/p'); do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V/librt_hip_$l.so; fi
  RT_EMU_FUSED=1 timeout -k 10 200 python scripts/rank_emulation.py 1 8 > gpurun_out/emu_$l.log 2>&1 || exit 1
  echo "${EMU_TAG:-cornell} $l N8 $(grep '^N=8' gpurun_out/emu_$l.log | sed 's/.*| max/max/') | N1 $(grep '^N=1' gpurun_out/emu_$l.log | sed 's/.*| max \([0-9.]*\).*/\1/')" | tee -a $out
done
done
unset RT_HIP_LIB
