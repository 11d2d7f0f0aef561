# interleaved A/B of every library variant in lib/variants against the main build (default
# bench, REPS rounds), then the GPU parity tests on each variant
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh ${REPS:-3} "$@" || exit 1
for f in mini-opencl-raytracer_amd/lib/variants/librt_hip_*.so; do
  v=$(basename $f .so); v=${v#librt_hip_}
  RT_HIP_LIB=$f timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fused_frames.py tests/test_benched_path.py tests/test_ref_opencl.py tests/test_wavefront.py -x -q --timeout 200 --timeout-method thread > gpurun_out/variant_tests_$v.log 2>&1
  echo "$v tests rc=$?"; tail -1 gpurun_out/variant_tests_$v.log
done
