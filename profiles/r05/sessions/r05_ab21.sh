# round-5 session 21: HBM/L2 node weight re-swept with node bursts of 5 (bunny), and the emulated ranks
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py tests/test_proxy_scene.py tests/test_benched_path.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab20_tests.txt 2>&1 || { tail -30 gpurun_out/ab20_tests.txt; exit 1; }
tail -1 gpurun_out/ab20_tests.txt
rm -f gpurun_out/sweep_goct_w4.txt
bash scripts/sweep.sh goct_w4 3 "step_weight_node_global=65" "step_weight_node_global=80" "step_weight_node_global=100" "step_weight_node_global=130" -- --scene bunny --no-drop-in || exit 1


