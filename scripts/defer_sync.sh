set -u
for rep in 1 2; do
for d in 0 1 2; do
  timeout -k 10 120 python scripts/perframe_loop.py --no-readback --tune perframe_defer=$d || exit 1
  timeout -k 10 120 python scripts/perframe_loop.py --tune perframe_defer=$d || exit 1
  timeout -k 10 120 python scripts/perframe_loop.py --scene bunny --no-readback --tune perframe_defer=$d || exit 1
  for cfg in "--width 1920 --height 1080 --bounces 2 --frames 1 --steps 20" "--width 512 --height 512 --bounces 1 --frames 1 --steps 50"; do
    timeout -k 10 120 python bench.py $cfg --no-cpu-baseline --tune perframe_defer=$d > gpurun_out/ds.json 2>&1 || exit 1
    python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/ds.json') if l.startswith('{')][-1])
print('bench ${cfg// /_} defer=$d', d['ms_per_frame'])"
  done
done
done
