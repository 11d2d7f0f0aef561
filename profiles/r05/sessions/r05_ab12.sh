# round-5 A/B session 12: pixel-major order as the default on HBM/L2 scenes (main) against the build
# before (headref): parity tests, bunny 3 rounds, emulated ranks (bunny) with the order forced at N = 8
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py tests/test_proxy_scene.py tests/test_benched_path.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab12_tests.txt 2>&1 || { tail -30 gpurun_out/ab12_tests.txt; exit 1; }
tail -2 gpurun_out/ab12_tests.txt
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --no-drop-in --scene bunny || exit 1
unset RT_HIP_LIB
for t in -1 2; do
  RT_EMU_SCENE=bunny RT_EMU_TUNE=tile_major=$t timeout -k 10 300 python scripts/rank_emulation.py 1 8 > gpurun_out/emu12_$t.txt 2>&1 || exit 1
  echo "== bunny tile_major=$t"; tail -2 gpurun_out/emu12_$t.txt
done
