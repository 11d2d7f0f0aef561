#!/bin/bash
# A/B the library variants in lib/variants/ (and the main build) on the default devicelib bench,
# interleaved and repeated.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
for v in mini-opencl-raytracer_amd/lib/variants/*.so main; do
  n=$(basename $v .so)
  if [ $v = main ]; then L=""; else L="RT_HIP_LIB=$v"; fi
  env $L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/abd_$n.log 2>&1 || exit $?
  echo "$n $(grep ms_per gpurun_out/abd_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_frame"])')" | tee -a gpurun_out/ab_dl.txt
done; done
