#!/bin/bash
# Threshold sweep of the step schedule (env overrides read by rtCreateKernel).
set -u
mkdir -p gpurun_out
for m in devicelib pinned; do
for r in 8 16 24 32 48; do for s in 8 16 24 32 48; do
  out=$(RT_REFILL_MIN=$r RT_SHADE_MIN=$s timeout -k 10 120 python bench.py --math $m --no-cpu-baseline --steps 3 --warmup 1) || exit $?
  echo "$m refill=$r shade=$s $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')"
done; done; done | tee gpurun_out/sweep.txt
