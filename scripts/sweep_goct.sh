# refill / shade thresholds of the octant walk over HBM/L2 (bunny proxy), ms/frame and render ms
set -u
mkdir -p gpurun_out
out=gpurun_out/sweep_goct.txt; rm -f $out
for tn in "" "refill_min_global=8" "refill_min_global=12" "refill_min_global=24" "shade_min_global=44" "shade_min_global=52" "step_weight_node=45"; do
  args=""; for x in $tn; do args="$args --tune $x"; done
  timeout -k 10 120 python bench.py --scene bunny --no-cpu-baseline --steps 6 $args > gpurun_out/sg.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sg.json') if l.startswith('{')][-1])
print('${tn:-default}', d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a $out
done
