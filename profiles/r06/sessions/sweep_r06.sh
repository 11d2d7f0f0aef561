set -u
bash scripts/sweep.sh cornell6 2 "" "shade_min=44" "shade_min=52" "refill_min=4" "refill_min=8" "step_weight_node=30" "step_weight_node=40" "step_weight_leaf=62" || exit 1
bash scripts/sweep.sh p1080 2 "" "perframe_defer_min=1000000" "refill_min=4" "refill_min=8" "shade_min=40" "tail_chunk=128" -- --width 1920 --height 1080 --bounces 2 --frames 1 || exit 1
bash scripts/sweep.sh bunny6 2 "" "refill_min_global=24" "refill_min_global=40" "shade_min_global=44" "shade_min_global=52" "step_weight_node_global=55" "step_weight_node_global=75" -- --scene bunny || exit 1
