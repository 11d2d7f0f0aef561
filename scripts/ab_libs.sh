#!/bin/bash
# Interleaved A/B of library builds and env settings on one bench config (ms/frame).
# usage: scripts/ab_libs.sh "BENCH ARGS" "label:ENV=v,ENV=v" ...   (RT_HIP_LIB=path selects a build)
set -u
mkdir -p gpurun_out
args=$1; shift
for rep in 1 2 3; do
  for cfg in "$@"; do
    label=${cfg%%:*}; vars=${cfg#*:}
    out=$(env $(echo $vars | tr ',' ' ') timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 $args) || exit $?
    echo "$label [$args] $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')"
  done
done | tee -a gpurun_out/ab_libs.txt
