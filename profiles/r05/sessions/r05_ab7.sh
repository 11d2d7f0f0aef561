# round-5 A/B session 7: 6 waves per SIMD on the LDS walk (80 VGPRs, spilling) with the fused rings shrunk so
# that 6 workgroups fit a CU's LDS (occ6ring) against main; default bench and the emulated ranks
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_quick.txt
timeout -k 10 300 python -u -m pytest tests/test_fused_frames.py -x -q -m gpu --timeout 120 --timeout-method thread -k "fused_equals or band or sequences" > gpurun_out/ab7_tests.txt 2>&1 || true
bash scripts/ab_quick.sh 3 --no-drop-in || exit 1
for l in main occ6ring; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  timeout -k 10 200 python scripts/rank_emulation.py 1 8 > gpurun_out/emu7_$l.txt 2>&1 || exit 1
  echo "== $l"; tail -2 gpurun_out/emu7_$l.txt
done
