set -o pipefail
bash scripts/sweep.sh thr_cornell 2 "" "refill_min=4" "refill_min=8" "shade_min=40" "shade_min=48" "step_weight_node=30" "step_weight_node=40" "step_weight_leaf=48" "step_weight_leaf=62" || exit 1
bash scripts/sweep.sh thr_bunny 2 "" "refill_min_global=12" "refill_min_global=24" "shade_min_global=40" "shade_min_global=56" -- --scene bunny || exit 1
rm -f gpurun_out/ab_quick.txt; bash scripts/ab_quick.sh 3 || exit 1
