set -u
for l in pc1 pc2; do
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so timeout -k 10 600 python -u -m pytest tests/test_benched_path.py tests/test_fused_frames.py tests/test_ref_runtime_build.py tests/test_ref_opencl.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pc_tests_$l.txt 2>&1; echo "$l tests rc=$? $(tail -1 gpurun_out/pc_tests_$l.txt)"
done
AB_CONFIGS="cornell;bunny --scene bunny;c2 --width 1920 --height 1080 --bounces 2 --frames 1 --steps 40" bash scripts/ab_session.sh 3
