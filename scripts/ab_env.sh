#!/bin/bash
# A/B of run-time switches on the default bench: scripts/ab_env.sh "<env A>" "<env B>" [bench args...]
# prints ms/frame and KernelEntry ms per launch, alternating A and B three times.
set -u
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for rep in 1 2 3; do
  for e in "$A" "$B"; do
    out=$(env $e timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@") || exit $?
    echo "[$e] $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"], d["roofline"]["kernel_ms"])')"
  done
done
