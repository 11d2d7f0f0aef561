# step-schedule thresholds after the chunking change; SCENE=bunny uses the *_global keys
set -u
mkdir -p gpurun_out
sc=${SCENE:-cornell}; out=gpurun_out/sweep_thr_$sc.txt; rm -f $out
if [ $sc = bunny ]; then R=refill_min_global; S=shade_min_global; else R=refill_min; S=shade_min; fi
for rep in 1 2; do
for tn in "" "$R=4" "$R=8" "$R=12" "$R=16" "$R=24" "$S=40" "$S=48" "$S=52" "step_weight_node=30" "step_weight_node=40" "step_weight_leaf=48" "step_weight_leaf=62"; do
  args=""; for x in $tn; do args="$args --tune $x"; done
  timeout -k 10 120 python bench.py --scene $sc --no-cpu-baseline --steps 10 $args > gpurun_out/sc.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sc.json') if l.startswith('{')][-1])
print('${tn:-default}', d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a $out
done; done
