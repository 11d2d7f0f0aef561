# round-5 session 27 (bunny): six waves per SIMD on the octant walk (goct6) against five, and the HBM/L2 shade
# threshold re-swept on the final defaults
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_quick.txt gpurun_out/sweep_goct_shade.txt
bash scripts/ab_quick.sh 3 --no-drop-in --scene bunny || exit 1
unset RT_HIP_LIB
bash scripts/sweep.sh goct_shade 2 "" "shade_min_global=44" "shade_min_global=52" -- --scene bunny --no-drop-in || exit 1
