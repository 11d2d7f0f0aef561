# round-5 session 15 (diagnostic): phase counters of the LDS walk with pixel-major ray-ring fills (ringpx)
# against main -- lanes per node / triangle step, shading batches, refills
set -u
mkdir -p gpurun_out
for l in main ringpx; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  RT_PHASE_MATH=shipped RT_PHASE_LB=9 RT_PHASE_TUNE=tile_major=2 timeout -k 10 300 python scripts/phase_profile.py > gpurun_out/phase15_$l.txt 2>&1 || exit 1
  echo "== $l"; cat gpurun_out/phase15_$l.txt
done
