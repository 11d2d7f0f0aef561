# round-5 A/B session 5: the world-1 gather flow (copy-ipc) with more hardware queues per process
# (GPU_MAX_HW_QUEUES 8 / 16 instead of HIP's default 4), main build and the 4-copy-stream variant
set -u
DIST_TAG=hwq DIST_LIBS="main xfer4" DIST_ENVS="hwq8:GPU_MAX_HW_QUEUES=8 hwq16:GPU_MAX_HW_QUEUES=16" \
  bash scripts/dist_ab.sh 2 --transport copy-ipc || exit 1
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_xfer4.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-drop-in --steps 20 --warmup 2 --force-dist --check-gather --transport copy-ipc > gpurun_out/dist_ab_hwq/xfer4_hwq$q.json 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/dist_ab_hwq/xfer4_hwq$q.json') if l.startswith('{')][-1])
print('xfer4 hwq$q', d['ms_per_frame'], d['roofline'].get('launch_ms'), d.get('check_gather', ''))"
done
