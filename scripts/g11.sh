set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_g11.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/pytest_gpu_g11.log
out=gpurun_out/g11.txt
rm -f $out
b() { local lab=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/g11.json 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/g11.json; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/g11.json') if l.startswith('{')][-1])
print('$lab', d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a $out; }
b cornell_step
b bunny_step --scene bunny --steps 5
b bunny_wf --scene bunny --steps 5 --sched wavefront
b bunny_step_r20 --scene bunny --steps 5 --tune refill_min_global=20
b bunny_step_r24 --scene bunny --steps 5 --tune refill_min_global=24
b bunny_step_w45 --scene bunny --steps 5 --tune step_weight_node=45
b bunny_step_tm0 --scene bunny --steps 5 --tune tile_major=0
