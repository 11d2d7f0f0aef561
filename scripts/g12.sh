set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_frames.py tests/test_proxy_scene.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_g12.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/pytest_g12.log
out=gpurun_out/g12.txt; rm -f $out
b() { local lab=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/g12.json 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/g12.json; exit 1; }
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/g12.json') if l.startswith('{')][-1])
print('$lab', d['ms_per_frame'], d['roofline']['launch_ms'])" | tee -a $out; }
for rep in 1 2; do
for t in 0 64 96; do b top$t --scene bunny --steps 5 --tune goct_top_nodes=$t; done
done
