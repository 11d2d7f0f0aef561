# step-schedule thresholds on the LDS scene path (4K Cornell fused), ms/frame and render ms, 2 rounds
set -u
mkdir -p gpurun_out
out=gpurun_out/sweep_cornell.txt; rm -f $out
for rep in 1 2; do
for tn in "" "refill_min=4" "refill_min=8" "refill_min=12" "shade_min=40" "shade_min=48" "shade_min=52" \
          "step_weight_node=30" "step_weight_node=40" "step_weight_leaf=48" "step_weight_leaf=62" \
          "chunk_pixels=64" "chunk_pixels=256"; do
  args=""; for x in $tn; do args="$args --tune $x"; done
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 $args > gpurun_out/sc.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sc.json') if l.startswith('{')][-1])
print('${tn:-default}', d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a $out
done
done
