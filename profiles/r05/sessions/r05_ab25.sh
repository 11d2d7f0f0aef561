# round-5 session 25: bulk chunks of 1024 in the pixel-major order (new auto) -- parity tests, bunny bench 3 rounds
# against chunk_pixels=512 forced, emulated ranks (bunny)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py tests/test_proxy_scene.py tests/test_benched_path.py tests/test_comm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab25_tests.txt 2>&1 || { tail -30 gpurun_out/ab25_tests.txt; exit 1; }
tail -1 gpurun_out/ab25_tests.txt
rm -f gpurun_out/sweep_goct_chunk2.txt
bash scripts/sweep.sh goct_chunk2 3 "" "chunk_pixels=512" "chunk_pixels=2048" -- --scene bunny --no-drop-in || exit 1
for c in 0 512; do
  RT_EMU_SCENE=bunny RT_EMU_TUNE=chunk_pixels=$c timeout -k 10 300 python scripts/rank_emulation.py 1 8 > gpurun_out/emu25_$c.txt 2>&1 || exit 1
  echo "== chunk_pixels=$c"; tail -2 gpurun_out/emu25_$c.txt
done
