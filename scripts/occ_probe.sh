# Occupancy probe: the persistent grid capped at 2..5 workgroups (x4 waves) per CU (RT_TUNE_MAX_BLOCKS):
# how much a scene path's time depends on the waves per SIMD (latency-bound: strongly)
set -o pipefail
bash scripts/sweep.sh occ_bunny 2 "" "max_blocks=4" "max_blocks=3" "max_blocks=2" -- --scene bunny || exit 1
bash scripts/sweep.sh occ_cornell 2 "" "max_blocks=4" "max_blocks=3" "max_blocks=2" || exit 1
