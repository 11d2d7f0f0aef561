# A/B of library variants on the fused rank emulation (N=1 and 8) for both scenes, plus the default bench
set -u
mkdir -p gpurun_out/abemu
rm -f gpurun_out/ab_quick.txt gpurun_out/abemu/summary.txt
bash scripts/ab_quick.sh 2 || exit 1
V=mini-opencl-raytracer_amd/lib/variants
for sc in cornell bunny; do
for l in main $(ls $V | sed -n 's/^librt_hip_\(.*\)\.so$/\1/p'); do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V/librt_hip_$l.so; fi
  RT_EMU_FUSED=1 RT_EMU_SCENE=$sc timeout -k 10 300 python scripts/rank_emulation.py 1 8 > gpurun_out/abemu/${sc}_$l.txt 2>&1 || exit 1
  echo "$sc $l $(grep -o 'max [0-9.]* | render-only strong-scaling efficiency [0-9.]*' gpurun_out/abemu/${sc}_$l.txt | tr '\n' ' ')" | tee -a gpurun_out/abemu/summary.txt
done; done
