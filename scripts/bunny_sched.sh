#!/bin/bash
# Bunny: step vs pool schedule (with / without top-of-tree LDS staging).
set -u
mkdir -p gpurun_out
run() { local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --scene bunny --no-cpu-baseline --steps 3 > gpurun_out/bs_$label.log 2>&1 || exit $?
  echo "$label $(grep ms_per gpurun_out/bs_$label.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')" | tee -a gpurun_out/bunny_sched.txt; }
run step X=1
run pool_top0 RT_SCHED=3 RT_TOP_NODES=0
run pool_top128 RT_SCHED=3 RT_TOP_NODES=128
run pool_top256 RT_SCHED=3
