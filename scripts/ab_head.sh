# main build vs variants (e.g. the previous commit's library) on bunny fused / per-frame and Cornell fused
set -o pipefail
V=mini-opencl-raytracer_amd/lib/variants
for rep in 1 2; do
  for l in main $(ls $V | sed -n 's/^librt_hip_\(.*\)\.so$/\1/p'); do
    if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V/librt_hip_$l.so; fi
    for cfg in "bunny fused" "bunny per-frame" "cornell fused"; do
      set -- $cfg
      timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 --scene $1 --launch $2 > gpurun_out/abh.json 2>&1 || exit 1
      python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/abh.json') if l.startswith('{')][-1]); print('$l $1 $2', d['ms_per_frame'])" | tee -a gpurun_out/ab_head.txt
    done
  done
done
