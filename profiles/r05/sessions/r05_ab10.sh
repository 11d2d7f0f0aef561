# round-5 A/B session 10: LDS-walk node visits without a per-visit exec branch (nobranch) against main:
# parity tests on the variant, default bench 3 rounds, emulated ranks
set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_nobranch.so timeout -k 10 900 python -u -m pytest tests/test_fused_frames.py tests/test_gpu_parity.py tests/test_benched_path.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab10_tests.txt 2>&1 || { tail -30 gpurun_out/ab10_tests.txt; exit 1; }
tail -2 gpurun_out/ab10_tests.txt
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --no-drop-in || exit 1
