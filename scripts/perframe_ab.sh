# Per-frame (drop-in) launch modes, 4K Cornell 9 bounces: queued back to back (bench.py --launch
# per-frame), and the reference's RenderFrame loop with rtFinish only / with the image read-back
# (scripts/perframe_loop.py); in-render accumulation (0), always deferred (1), automatic (2)
set -o pipefail
for rep in 1 2; do
  for d in 0 1 2; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-drop-in --launch per-frame --steps 5 --tune perframe_defer=$d > gpurun_out/pf_$d.json || exit 1
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/pf_$d.json') if l.startswith('{')][-1]); print('queued defer=$d', d['ms_per_frame'])"
    timeout -k 10 120 python scripts/perframe_loop.py --tune perframe_defer=$d --no-readback || exit 1
    timeout -k 10 120 python scripts/perframe_loop.py --tune perframe_defer=$d || exit 1
  done
done
