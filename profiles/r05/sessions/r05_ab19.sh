# round-5 A/B session 19: octant-walk node bursts 4 (main) / 5 / 6 / 8 with the HBM/L2 step weights 45 / 55 (new
# default), and main with the old weight 35 (sweep); parity tests on onb6
set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_onb6.so timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py tests/test_proxy_scene.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab19_tests.txt 2>&1 || { tail -30 gpurun_out/ab19_tests.txt; exit 1; }
tail -1 gpurun_out/ab19_tests.txt
rm -f gpurun_out/ab_quick.txt gpurun_out/sweep_goct_w2.txt
bash scripts/ab_quick.sh 3 --no-drop-in --scene bunny || exit 1
bash scripts/sweep.sh goct_w2 2 "" "step_weight_node_global=35" "step_weight_node_global=55" -- --scene bunny --no-drop-in || exit 1
