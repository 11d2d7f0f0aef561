#!/bin/bash
# Env-override sweep of the default bench: each argument is "LABEL:VAR=v,VAR=v".
# usage: scripts/sweep_env.sh MATH "a:RT_SHADE_MIN=40" "b:RT_REFILL_MIN=8,RT_SHADE_MIN=56" ...
set -u
mkdir -p gpurun_out
m=$1; shift
for cfg in "$@"; do
  label=${cfg%%:*}; vars=${cfg#*:}
  out=$(env $(echo $vars | tr ',' ' ') timeout -k 10 120 python bench.py --math $m --no-cpu-baseline --steps 3 --warmup 1) || exit $?
  echo "$m $label $vars $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')"
done | tee -a gpurun_out/sweep_env_$m.txt
