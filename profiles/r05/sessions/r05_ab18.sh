# round-5 A/B session 18: the HBM/L2 walk's step weights and bursts re-tuned under the pixel-major order (bunny)
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_quick.txt gpurun_out/sweep_goct_w.txt
bash scripts/ab_quick.sh 2 --no-drop-in --scene bunny || exit 1
bash scripts/sweep.sh goct_w 2 "" "step_weight_node=45" "step_weight_node=25" "step_weight_leaf=45" "step_weight_leaf=70" -- --scene bunny --no-drop-in || exit 1
