#!/bin/bash
# One A/B round of library variants (scripts/build_variant.sh) against the main build on one GPU:
# parity tests on the main build, then bench.py (fused 4K 8 spp; Cornell, bunny proxy, Cornell
# per-frame launches) and the emulated N = 8 rank step for every library, REPS rounds.
# usage: scripts/ab_round.sh [REPS]   -> gpurun_out/ab_round.txt
set -o pipefail
reps=${1:-2}
O=gpurun_out/ab_round.txt; : > $O
timeout -k 10 400 python -u -m pytest tests/test_benched_path.py tests/test_fused_frames.py tests/test_comm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_round_tests.log 2>&1 || { tail -30 gpurun_out/ab_round_tests.log; exit 1; }
tail -1 gpurun_out/ab_round_tests.log | tee -a $O
V=mini-opencl-raytracer_amd/lib/variants
for rep in $(seq $reps); do
  for l in main $(ls $V 2>/dev/null | sed -n 's/^librt_hip_\(.*\)\.so$/\1/p'); do
    if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=$V/librt_hip_$l.so; fi
    for cfg in "cornell fused" "bunny fused" "cornell per-frame"; do
      set -- $cfg
      timeout -k 10 120 python bench.py --no-cpu-baseline --no-configs --steps 10 --scene $1 --launch $2 > gpurun_out/ab_last.json 2>&1 || exit 1
      python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/ab_last.json') if l.startswith('{')][-1])
print('$l', '$1', '$2', 'ms/frame', d['ms_per_frame'])" | tee -a $O
    done
    for sc in cornell bunny; do
      RT_EMU_FUSED=1 RT_EMU_SCENE=$sc RT_EMU_STEPS=10 timeout -k 10 120 python scripts/rank_emulation.py 8 > gpurun_out/ab_emu.txt 2>&1 || exit 1
      echo "$l $sc N=8 max rank ms/step $(grep -o 'max [0-9.]*' gpurun_out/ab_emu.txt)" | tee -a $O
    done
  done
done
unset RT_HIP_LIB
