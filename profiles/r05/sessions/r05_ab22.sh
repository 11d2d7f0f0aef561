# round-5 A/B session 22 (bunny, pixel-major order, bursts 5, weights 65/55): triangle bursts 1 / 3 (main 2),
# record groups of 2 / 4 nodes (main 1), then the HBM/L2 refill / shade thresholds re-swept
set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_grp2.so timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py tests/test_proxy_scene.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab22_tests.txt 2>&1 || { tail -30 gpurun_out/ab22_tests.txt; exit 1; }
tail -1 gpurun_out/ab22_tests.txt
rm -f gpurun_out/ab_quick.txt gpurun_out/sweep_goct_thr2.txt
bash scripts/ab_quick.sh 2 --no-drop-in --scene bunny || exit 1
unset RT_HIP_LIB
bash scripts/sweep.sh goct_thr2 2 "" "refill_min_global=24" "refill_min_global=32" "shade_min_global=40" "shade_min_global=56" -- --scene bunny --no-drop-in || exit 1
