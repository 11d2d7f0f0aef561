# round-5 session 14: the HBM/L2 walk's load coherence under the pixel-major order (8 fused frames), and its
# thresholds re-swept
set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/diag/librt_hip_lds_conflicts.so timeout -k 10 300 python scripts/goct_coherence.py 8 > gpurun_out/goct_coherence_px.txt 2>&1 || exit 1
cat gpurun_out/goct_coherence_px.txt
rm -f gpurun_out/sweep_goct_px.txt
bash scripts/sweep.sh goct_px 2 "" "shade_min_global=40" "shade_min_global=56" "refill_min_global=12" "refill_min_global=24" -- --scene bunny --no-drop-in || exit 1
