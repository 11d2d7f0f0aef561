#!/bin/bash
# N = 8 rank emulation (fused 4K 8 spp) over the tail-chunk cap, both scenes
set -u
mkdir -p gpurun_out/n8tail
for sc in cornell bunny; do
  for tc in 256 128 64; do
    echo "== scene=$sc tail_chunk=$tc" >> gpurun_out/n8tail/sweep.txt
    RT_EMU_FUSED=1 RT_EMU_SCENE=$sc RT_EMU_TUNE=tail_chunk=$tc timeout -k 10 120 \
      python scripts/rank_emulation.py 1 8 >> gpurun_out/n8tail/sweep.txt 2>&1 || exit 1
  done
done
cat gpurun_out/n8tail/sweep.txt
