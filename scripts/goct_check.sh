set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_frames.py -k "global_octant" -x -v --timeout 120 --timeout-method thread > gpurun_out/goct_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/goct_tests.log
for rep in 1 2; do
for t in 0 1; do
  timeout -k 10 120 python bench.py --scene bunny --no-cpu-baseline --steps 5 --tune global_oct=$t > gpurun_out/goct_$t.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/goct_$t.json') if l.startswith('{')][-1])
print('global_oct=$t', d['ms_per_frame'], d['roofline']['launch_ms'])"
done
done
