# round-5 A/B session 9: scalar-cache reads for steps whose lanes read one of TWO records (scalar2) against
# the shipped one-record rule (main): global-scene parity tests, bunny bench 3 rounds, address-unit counters
set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_scalar2.so timeout -k 10 900 python -u -m pytest tests/test_fused_frames.py tests/test_proxy_scene.py tests/test_benched_path.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab9_tests.txt 2>&1 || { tail -30 gpurun_out/ab9_tests.txt; exit 1; }
tail -2 gpurun_out/ab9_tests.txt
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --no-drop-in --scene bunny || exit 1
for l in main scalar2; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  timeout -s KILL 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ta9_$l -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for l in ("main", "scalar2"):
    acc = defaultdict(list)
    for f in glob.glob(f'gpurun_out/ta9_{l}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'goct' in r['Kernel_Name']:
                acc[r['Counter_Name']].append((int(r['Dispatch_Id']), float(r['Counter_Value'])))
    print(l, {k: [round(x[1] / 1e6, 2) for x in sorted(v)] for k, v in acc.items()})
PY
