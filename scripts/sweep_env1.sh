#!/bin/bash
# sweep one run-time knob on the default bench: scripts/sweep_env1.sh VAR "v1 v2 ..." [bench args...]
set -u
VAR=$1; VALS=$2; shift 2
for rep in 1 2; do
  for v in $VALS; do
    out=$(env $VAR=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@") || exit $?
    echo "$VAR=$v $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"], d["roofline"]["kernel_ms"])')"
  done
done
