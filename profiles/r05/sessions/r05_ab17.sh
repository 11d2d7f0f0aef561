# round-5 A/B session 17: pixel-major order with the unit's 8 pixels as a 2 x 4 block (pxquad)
# against a tile row (main): parity tests on each variant, bunny bench 3 rounds
set -u
mkdir -p gpurun_out
for l in pxquad; do
  RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py -x -q -m gpu --timeout 300 --timeout-method thread -k "pixel_major or global or bunny" > gpurun_out/ab16_tests_$l.txt 2>&1 || { tail -30 gpurun_out/ab16_tests_$l.txt; exit 1; }
  tail -1 gpurun_out/ab16_tests_$l.txt
done
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --no-drop-in --scene bunny || exit 1
