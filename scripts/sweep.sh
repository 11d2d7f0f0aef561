#!/bin/bash
# Sweep library tunings (rt_hip.h RT_TUNE_*, every value renders the same bits) on bench.py:
#   scripts/sweep.sh NAME REPS "SET" ["SET" ...] [-- BENCH_ARGS...]
# Each SET is a space-separated list of name=value tunings ("" = the defaults); every set runs
# once per round, REPS rounds interleaved.  Prints and appends to gpurun_out/sweep_NAME.txt:
#   set | ms per frame | render launch ms
# e.g. scripts/sweep.sh thr 2 "" "refill_min=8" "shade_min=40 refill_min=4" -- --scene bunny
set -u
name=$1; reps=$2; shift 2
sets=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
mkdir -p gpurun_out
out=gpurun_out/sweep_$name.txt
for rep in $(seq $reps); do
  for set in "${sets[@]}"; do
    args=""; for x in $set; do args="$args --tune $x"; done
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-drop-in --no-configs --steps 10 $args "$@" > gpurun_out/sweep_last.json 2>&1 || exit 1
    python3 - "$set" <<'PY' | tee -a $out
import json, sys
d = json.loads([l for l in open('gpurun_out/sweep_last.json') if l.startswith('{')][-1])
r = d["roofline"]
print(f"{sys.argv[1] or 'defaults':40s} {d['ms_per_frame']:.4f} {r.get('launch_ms', r.get('kernel_ms'))}")
PY
  done
done
