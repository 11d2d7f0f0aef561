# round-5 session 23 (bunny): HBM/L2 refill threshold 16 (default) / 32 / 40 / 48, and record groups of 2 with 32
set -u
mkdir -p gpurun_out
rm -f gpurun_out/sweep_goct_thr3.txt gpurun_out/ab_quick.txt
bash scripts/sweep.sh goct_thr3 3 "" "refill_min_global=32" "refill_min_global=40" "refill_min_global=48" -- --scene bunny --no-drop-in || exit 1
bash scripts/ab_quick.sh 3 --no-drop-in --scene bunny --tune refill_min_global=32 || exit 1
