# round-5 A/B session 11: pixel-major work order on the HBM/L2 walk (tile_major 2: a unit is one tile row
# x the 8 frames) against the default tile-major order, and the build before the change (headref):
# parity tests, bunny sweep 3 rounds, coherence of the walk under both orders
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab11_tests.txt 2>&1 || { tail -30 gpurun_out/ab11_tests.txt; exit 1; }
tail -2 gpurun_out/ab11_tests.txt
rm -f gpurun_out/sweep_pxmajor.txt
for rep in 1 2 3; do
  RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_headref.so timeout -k 10 120 python bench.py --scene bunny --no-cpu-baseline --no-drop-in --steps 10 > gpurun_out/sweep_last.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sweep_last.json') if l.startswith('{')][-1])
print('headref', d['ms_per_frame'], d['roofline'].get('launch_ms'), d['roofline'].get('ta_busy'))" | tee -a gpurun_out/sweep_pxmajor.txt
  for t in -1 2; do
    timeout -k 10 120 python bench.py --scene bunny --no-cpu-baseline --no-drop-in --steps 10 --tune tile_major=$t > gpurun_out/sweep_last.json 2>&1 || exit 1
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/sweep_last.json') if l.startswith('{')][-1])
print('main tile_major=$t', d['ms_per_frame'], d['roofline'].get('launch_ms'))" | tee -a gpurun_out/sweep_pxmajor.txt
  done
done
