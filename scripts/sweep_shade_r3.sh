set -o pipefail
bash scripts/sweep.sh shade_c 3 "" "shade_min=46" "shade_min=48" "shade_min=50" "shade_min=52" || exit 1
bash scripts/sweep.sh shade_pf 2 "" "shade_min=48" "shade_min=52" -- --launch per-frame || exit 1
