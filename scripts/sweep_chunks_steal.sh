set -o pipefail
bash scripts/sweep.sh chunks_c 2 "" "tail_chunk=512" "tail_chunk=1024" "chunk_pixels=1024" "chunk_pixels=1024 tail_chunk=512" "bulk_percent=90" "bulk_percent=100" || exit 1
for t in "" "tail_chunk=512" "tail_chunk=1024" "chunk_pixels=1024" "bulk_percent=90" "bulk_percent=100"; do
  tt=$(echo $t | tr ' ' ',')
  RT_EMU_FUSED=1 RT_EMU_STEPS=10 RT_EMU_TUNE=$tt timeout -k 10 120 python scripts/rank_emulation.py 8 > gpurun_out/emu_sw.txt 2>&1 || exit 1
  echo "N8 cornell [$t] $(grep -o 'max [0-9.]*' gpurun_out/emu_sw.txt)" | tee -a gpurun_out/sweep_chunks_c.txt
done
