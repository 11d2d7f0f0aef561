#!/bin/bash
# N = 8 rank emulation (fused, 4K 8 spp) over the bulk share and bulk chunk size
set -u
mkdir -p gpurun_out/n8sweep
sc=${1:-cornell}
for cp in 512 256 128; do
  for bp in 80 60 40 0; do
    echo "== scene=$sc chunk_pixels=$cp bulk_percent=$bp" >> gpurun_out/n8sweep/$sc.txt
    RT_EMU_FUSED=1 RT_EMU_SCENE=$sc RT_EMU_TUNE=chunk_pixels=$cp,bulk_percent=$bp timeout -k 10 120 \
      python scripts/rank_emulation.py 8 >> gpurun_out/n8sweep/$sc.txt 2>&1 || exit 1
  done
done
