# round-5 session 28 (bunny): bulk share 80 % (default) vs 90 % with the pixel-major chunks of 1024, and the N = 8 rank
set -u
mkdir -p gpurun_out
rm -f gpurun_out/sweep_goct_bulk.txt
bash scripts/sweep.sh goct_bulk 3 "" "bulk_percent=90" -- --scene bunny --no-drop-in || exit 1
for b in 80 90; do
  RT_EMU_SCENE=bunny RT_EMU_TUNE=bulk_percent=$b timeout -k 10 300 python scripts/rank_emulation.py 1 8 > gpurun_out/emu28_$b.txt 2>&1 || exit 1
  echo "== bulk $b"; tail -2 gpurun_out/emu28_$b.txt
done
