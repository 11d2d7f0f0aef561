#!/bin/bash
# Threshold sweep of the pool schedule (env overrides read by rtCreateKernel).
set -u
mkdir -p gpurun_out
m=${1:-devicelib}
run() {  # run <label> <env...>
  out=$(env "${@:2}" timeout -k 10 120 python bench.py --math $m --sched pool --no-cpu-baseline --steps 3 --warmup 1) || exit $?
  echo "$m $1 $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')"
}
{
for p in 4 8 16 24 32; do run "park=$p" RT_PARK_MIN=$p; done
for r in 4 8 16 32; do run "refill=$r" RT_REFILL_MIN=$r; done
for l in 8 16 32 48 64; do run "low=$l" RT_LOW_WORK=$l; done
for s in 32 48 56; do run "shade=$s" RT_POOL_SHADE=$s; done
for w in "25 55" "35 45" "35 70" "45 55"; do set -- $w; run "w=$1/$2" RT_W_NODE=$1 RT_W_LEAF=$2; done
} | tee gpurun_out/sweep_pool_$m.txt
