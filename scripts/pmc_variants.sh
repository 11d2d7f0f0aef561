#!/bin/bash
# Counter groups of one bench command on the main build and on every library variant
# (mini-opencl-raytracer_amd/lib/variants, scripts/build_variant.sh; none = the main build only): one
# rocprofv3 --pmc pass per group and library, per-kernel sums printed by scripts/pmc_sum.py.
# usage: scripts/pmc_variants.sh "COUNTERS;COUNTERS;..." [bench args]
# (round 3 folded the one-off counter scripts into this one; scripts/README.md lists the group sets)
set -u
GROUPS_=$1; shift
export TMPDIR=/tmp
V=mini-opencl-raytracer_amd/lib/variants
for l in main $(ls $V 2>/dev/null | sed -n 's/^librt_hip_\(.*\)\.so$/\1/p'); do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V/librt_hip_$l.so; fi
  D=gpurun_out/pmcv_$l; rm -rf $D; mkdir -p $D
  i=0
  IFS=';' read -ra GS <<< "$GROUPS_"
  for g in "${GS[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $D/p_$i -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in "$@" > $D/p_$i.log 2>&1 || { echo "$l pass $i failed"; tail -5 $D/p_$i.log; exit 1; }
  done
  echo "== $l $*"
  python3 scripts/pmc_sum.py $D --all | grep -A12 "kernel_entry_step" | head -14
done
