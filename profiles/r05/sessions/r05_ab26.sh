# round-5 session 26 (Cornell, LDS walk): work-distribution knobs re-checked on the final build
set -u
mkdir -p gpurun_out
rm -f gpurun_out/sweep_lds_chunk.txt
bash scripts/sweep.sh lds_chunk 2 "" "chunk_pixels=1024" "chunk_pixels=256" "bulk_percent=90" "tail_chunk=128" -- --no-drop-in || exit 1
