# wavefront / global-path sweeps on the bunny proxy (ms/frame per line)
set -u
mkdir -p gpurun_out
out=gpurun_out/sweep_wf.txt
run() {  # run LABEL bench-args...
  local lab=$1; shift
  timeout -k 10 120 python bench.py --scene bunny --no-cpu-baseline --steps 4 "$@" > gpurun_out/sw.json 2>gpurun_out/sw.err || { echo "$lab FAILED"; tail -3 gpurun_out/sw.err; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sw.json') if l.startswith('{')][-1])
print('$lab', d['ms_per_frame'])" | tee -a $out
}
bash scripts/ab_quick.sh 2 --scene bunny
run step_top0 --tune top_nodes=0
run wf_default --sched wavefront
for v in 1 4 16 32; do run wf_refill$v --sched wavefront --tune wf_refill_min=$v; done
for v in 0 128 384; do run wf_top$v --sched wavefront --tune wf_top_nodes=$v; done
run wf_streams16 --sched wavefront --tune wf_streams_per_cu=16
run wf_framemajor --sched wavefront --tune tile_major=0
run wf_tilemajor --sched wavefront --tune tile_major=1
