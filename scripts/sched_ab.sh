#!/bin/bash
# Schedules side by side on the default bench (bench.py --sched), plus env variants of the pool.
set -u
mkdir -p gpurun_out
run() { local label=$1 sched=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --sched $sched --no-cpu-baseline --steps 3 > gpurun_out/sab_$label.log 2>&1 || exit $?
  echo "$label $(grep ms_per gpurun_out/sab_$label.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')" | tee -a gpurun_out/sched_ab.txt; }
run step step X=1
run pool pool X=1
run pool_p8 pool RT_PARK_MIN=8
run pool_p24 pool RT_PARK_MIN=24
run pool_low16 pool RT_LOW_WORK=16
run regen regen X=1
run tiles tiles X=1
