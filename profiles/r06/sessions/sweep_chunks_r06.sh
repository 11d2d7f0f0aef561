#!/bin/bash
# Round 6: bulk / tail chunk sizes after the small-launch hand-out change -- 4K fused Cornell (bench.py)
# and the emulated N = 8 fused rank (scripts/rank_emulation.py) per tuning set.
set -u
rm -f gpurun_out/sweep_chunks.txt
bash scripts/sweep.sh chunks 2 "" "chunk_pixels=1024" "chunk_pixels=2048" "tail_chunk=512" "bulk_percent=90" "chunk_pixels=1024 tail_chunk=512" || exit 1
O=gpurun_out/sweep_chunks_n8.txt; : > $O
for t in "" "chunk_pixels=1024" "chunk_pixels=2048" "tail_chunk=512" "bulk_percent=90" "chunk_pixels=1024,tail_chunk=512"; do
  RT_EMU_TUNE="$t" RT_EMU_FUSED=1 RT_EMU_SCENE=cornell RT_EMU_STEPS=10 timeout -k 10 300 python scripts/rank_emulation.py 8 > gpurun_out/sc_emu.txt 2>&1 || exit 1
  echo "${t:-defaults} $(grep -o 'max [0-9.]*' gpurun_out/sc_emu.txt)" | tee -a $O
done
