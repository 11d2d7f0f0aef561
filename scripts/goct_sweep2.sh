set -u
mkdir -p gpurun_out
out=gpurun_out/goct_sweep2.txt
for tn in "refill_min_global=8 shade_min_global=48" "refill_min_global=12 shade_min_global=48" "refill_min_global=16 shade_min_global=48" "refill_min_global=12 shade_min_global=44" "refill_min_global=12 shade_min_global=52" "refill_min_global=8 shade_min_global=48 tile_major=0" "refill_min_global=8 shade_min_global=48 step_weight_node=45" "refill_min_global=8 shade_min_global=48 step_weight_node=28"; do
  args=""; for x in $tn; do args="$args --tune $x"; done
  timeout -k 10 120 python bench.py --scene bunny --no-cpu-baseline --steps 5 --tune global_oct=1 $args > gpurun_out/gs.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/gs.json') if l.startswith('{')][-1])
print('$tn', d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a $out
done
