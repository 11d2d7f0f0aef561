#!/bin/bash
set -u
mkdir -p gpurun_out
for m in devicelib pinned; do
for wl in 1000 80 55 35 20; do
  out=$(RT_W_NODE=35 RT_W_LEAF=$wl timeout -k 10 120 python bench.py --math $m --no-cpu-baseline --steps 3 --warmup 1) || exit $?
  echo "$m wnode=35 wleaf=$wl $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')"
done; done | tee gpurun_out/sweep_w.txt
