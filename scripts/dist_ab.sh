#!/bin/bash
# The bench's N > 1 flow at world size 1 (RCCL communicator, pack / self-send / unpack every step,
# pipelined with the next step) against the same bench without the gather, for the main build and
# every library variant (lib/variants/librt_hip_*.so), REPS interleaved rounds; then one
# rocprofv3 kernel + memory-copy trace of the flow per build (scripts/stream_timeline.py reads it).
# usage: scripts/dist_ab.sh [REPS] [bench args...]
#   DIST_LIBS="main nocu ..."        a subset of the builds
#   DIST_ENVS="name:VAR=v,VAR2=w ..."  extra runs of the main build under environment settings
#                                      (e.g. RCCL's channel counts), named name
#   DIST_TAG=tag                       outputs under gpurun_out/dist_ab_tag
set -u
OUT=gpurun_out/dist_ab${DIST_TAG:+_$DIST_TAG}
mkdir -p $OUT
export TMPDIR=/tmp
reps=${1:-2}; shift || true
V=mini-opencl-raytracer_amd/lib/variants
libs=${DIST_LIBS:-"main $(ls $V 2>/dev/null | sed -n 's/^librt_hip_\(.*\)\.so$/\1/p')"}
envs=${DIST_ENVS:-}
run() {  # run <name> <args...>
  local name=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-drop-in --steps 20 --warmup 2 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "FAILED $name"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('$OUT/$name.json') if l.startswith('{')][-1])
print('$name', d['ms_per_frame'], d['roofline'].get('launch_ms'), d.get('check_gather', ''))" | tee -a $OUT/summary.txt
}
pick() {  # select <lib-or-envspec>: sets RT_HIP_LIB / the variables for one build
  unset RT_HIP_LIB
  case $1 in
    *:*) for kv in $(echo ${1#*:} | tr ',' ' '); do export "$kv"; done ;;
    main) ;;
    *) export RT_HIP_LIB=$V/librt_hip_$1.so ;;
  esac
}
unpick() { case $1 in *:*) for kv in $(echo ${1#*:} | tr ',' ' '); do unset "${kv%%=*}"; done ;; esac; }
for rep in $(seq $reps); do
  for l in $libs $envs; do
    n=${l%%:*}
    pick $l
    run ${n}_nodist_$rep "$@"
    run ${n}_dist_$rep --force-dist --check-gather "$@"
    unpick $l
  done
done
for l in $libs $envs; do
  n=${l%%:*}
  pick $l
  timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_$n -o run -- \
    python bench.py --no-cpu-baseline --no-drop-in --steps 5 --warmup 1 --force-dist "$@" > $OUT/trace_$n.log 2>&1 || { echo "trace $n failed"; tail -5 $OUT/trace_$n.log; exit 1; }
  python3 scripts/stream_timeline.py $OUT/trace_$n --last 60 > $OUT/timeline_$n.txt 2>&1
  tail -1 $OUT/timeline_$n.txt
  unpick $l
done
