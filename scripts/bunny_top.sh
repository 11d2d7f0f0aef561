#!/bin/bash
# Bunny (global-memory scene path): sweep the number of top-of-tree node records staged in LDS.
set -u
mkdir -p gpurun_out
for t in "$@"; do
  RT_TOP_NODES=$t timeout -k 10 200 python bench.py --scene bunny --no-cpu-baseline --steps 3 > gpurun_out/bunny_top$t.log 2>&1 || exit $?
  echo "top=$t $(grep ms_per gpurun_out/bunny_top$t.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')" | tee -a gpurun_out/bunny_top.txt
done
