#!/bin/bash
# One GPU A/B session (round 6): optional probe binaries, the parity tests of the main build, then
# every library variant under mini-opencl-raytracer_amd/lib/variants against the main build on the
# bench configurations named in AB_CONFIGS (scripts/ab_quick.sh), REPS interleaved rounds.
# usage: [AB_PROBES="scripts/probes/x ..."] [AB_TESTS="tests/a.py ..."] [AB_CONFIGS="cornell;bunny --scene bunny"] \
#        scripts/ab_session.sh [REPS]      -> gpurun_out/ab_session.txt
set -u
reps=${1:-3}
mkdir -p gpurun_out
O=gpurun_out/ab_session.txt; : > $O
for p in ${AB_PROBES:-}; do
  timeout -k 10 180 ./$p > gpurun_out/$(basename $p).txt 2>&1; rc=$?
  echo "== probe $p rc=$rc" | tee -a $O; cat gpurun_out/$(basename $p).txt | tee -a $O
  [ $rc -eq 0 ] || exit $rc
done
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${AB_TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.txt 2>&1; rc=$?
  echo "== tests rc=$rc: $(tail -1 gpurun_out/ab_tests.txt)" | tee -a $O
  [ $rc -eq 0 ] || { tail -30 gpurun_out/ab_tests.txt; exit 1; }
fi
IFS=';' read -ra CFGS <<< "${AB_CONFIGS:-cornell}"
for c in "${CFGS[@]}"; do
  set -- $c; name=$1; shift
  rm -f gpurun_out/ab_quick.txt
  bash scripts/ab_quick.sh $reps --no-drop-in --no-configs "$@" > /dev/null || exit 1
  echo "== $name ($*): variant ms/frame launch_ms" | tee -a $O
  sort gpurun_out/ab_quick.txt | tee -a $O
done
