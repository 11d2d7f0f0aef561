# after the chunking change: GPU tests, bench lines, fused rank emulation (new defaults vs round-1 chunking)
set -u
mkdir -p gpurun_out/chunk
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/chunk/pytest.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/chunk/pytest.log
for cfg in "" "--scene bunny" "--launch per-frame" "--scene bunny --launch per-frame" "--width 1920 --height 1080" "--width 512 --height 512"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline $cfg > gpurun_out/sc.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sc.json') if l.startswith('{')][-1])
print('${cfg:-default}', d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a gpurun_out/chunk/bench.txt
done
for sc in cornell bunny; do
  RT_EMU_FUSED=1 RT_EMU_SCENE=$sc timeout -k 10 400 python scripts/rank_emulation.py > gpurun_out/chunk/emu_$sc.txt 2>&1 || exit 1
  RT_EMU_FUSED=1 RT_EMU_SCENE=$sc RT_EMU_TUNE=chunk_pixels=128,tail_chunk=64 timeout -k 10 400 python scripts/rank_emulation.py > gpurun_out/chunk/emu_${sc}_r1chunks.txt 2>&1 || exit 1
done
