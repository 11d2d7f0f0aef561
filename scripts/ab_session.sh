set -u
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/probes/pinned_fast_probe > gpurun_out/pinned_fast_probe.txt 2>&1; echo "probe rc=$?"; cat gpurun_out/pinned_fast_probe.txt
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_dd.so timeout -k 10 600 python -u -m pytest tests/test_proxy_scene.py tests/test_benched_path.py -x -q -m gpu --timeout 300 --timeout-method thread -k "bunny or proxy" > gpurun_out/dd_tests.txt 2>&1; echo "dd tests rc=$?"; tail -3 gpurun_out/dd_tests.txt
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --scene bunny --no-drop-in --no-configs || exit 1
for l in main dd; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  timeout -s KILL 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ta_$l -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in --no-configs > /dev/null 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/sq_$l -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in --no-configs > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for l in ("main", "dd"):
    acc = defaultdict(list)
    for d in ("ta", "sq"):
        for f in glob.glob(f'gpurun_out/{d}_{l}/**/*counter_collection.csv', recursive=True):
            for r in csv.DictReader(open(f)):
                if 'goct' in r['Kernel_Name'] and '<false' in r['Kernel_Name']:
                    acc[r['Counter_Name']].append(float(r['Counter_Value']))
    e = {k: sum(v) / len(v) for k, v in acc.items()}
    print(l, {k: round(v / 1e6, 2) for k, v in e.items()},
          "ta_busy", round(e["TA_TA_BUSY_sum"] / 256 / (e["GRBM_GUI_ACTIVE"] / 8), 3),
          "lane_util", round(e["SQ_THREAD_CYCLES_VALU"] / 64 / e["SQ_INSTS_VALU"], 3),
          "wait", round(e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"], 3))
PY
