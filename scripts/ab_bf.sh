set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 || exit 1
for v in bfn bfnt; do
  RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fused_frames.py tests/test_benched_path.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bf_tests_$v.log 2>&1
  echo "$v tests rc=$?"; tail -1 gpurun_out/bf_tests_$v.log
done
