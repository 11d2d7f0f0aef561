# round-5 session 24 (bunny, final octant-walk defaults): work-distribution knobs re-checked, and the emulated ranks
set -u
mkdir -p gpurun_out
rm -f gpurun_out/sweep_goct_chunk.txt
bash scripts/sweep.sh goct_chunk 2 "" "chunk_pixels=1024" "chunk_pixels=256" "tail_chunk=128" "bulk_percent=70" "bulk_percent=90" -- --scene bunny --no-drop-in || exit 1
RT_EMU_SCENE=bunny timeout -k 10 300 python scripts/rank_emulation.py 1 8 > gpurun_out/emu24.txt 2>&1 || exit 1
tail -2 gpurun_out/emu24.txt
