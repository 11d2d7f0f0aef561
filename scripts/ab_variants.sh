#!/bin/bash
# A/B of experimental library builds (scripts/build_variant.sh) against the main build, on the
# default bench: ms/frame per variant, twice (interleaved), one bounded step each.
# usage: scripts/ab_variants.sh MATH [extra bench args...]
set -u
mkdir -p gpurun_out
m=$1; shift
one() {  # one <label> [env...]
  local label=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --math $m --no-cpu-baseline --steps 3 --warmup 1 "${EXTRA[@]}") || exit $?
  echo "$m $label $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"], d["roofline"]["kernel_ms"])')"
}
EXTRA=("$@")
for rep in 1 2; do
  one main RT_NONE=1
  for v in mini-opencl-raytracer_amd/lib/variants/*.so; do
    one $(basename $v .so) RT_HIP_LIB=$v
  done
done | tee -a gpurun_out/ab_variants_$m.txt
