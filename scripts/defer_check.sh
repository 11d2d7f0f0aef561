set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_frames.py -k "defer or sky or order or readback" -x -q --timeout 120 --timeout-method thread > gpurun_out/defer_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/defer_tests.log
for rep in 1 2; do
for d in 0 1 2; do
  for sc in cornell bunny; do
    timeout -k 10 200 python bench.py --launch per-frame --scene $sc --no-cpu-baseline --steps 5 --tune perframe_defer=$d > gpurun_out/df.json 2>&1 || exit 1
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/df.json') if l.startswith('{')][-1])
print('$sc per-frame defer=$d', d['ms_per_frame'])"
  done
done
done
