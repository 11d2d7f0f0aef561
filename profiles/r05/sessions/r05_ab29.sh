# round-5 A/B session 29 (bunny): shading records and materials read through the scalar cache when every lane of a
# shading round uses the same one (shadescalar) against main: parity tests on the variant, bunny 3 rounds, TA counters
set -u
mkdir -p gpurun_out
RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_shadescalar.so timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py tests/test_proxy_scene.py tests/test_benched_path.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab29_tests.txt 2>&1 || { tail -30 gpurun_out/ab29_tests.txt; exit 1; }
tail -1 gpurun_out/ab29_tests.txt
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --no-drop-in --scene bunny || exit 1
for l in main shadescalar; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  timeout -s KILL 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ta29_$l -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for l in ("main", "shadescalar"):
    acc = defaultdict(list)
    for f in glob.glob(f'gpurun_out/ta29_{l}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'goct' in r['Kernel_Name']:
                acc[r['Counter_Name']].append((int(r['Dispatch_Id']), float(r['Counter_Value'])))
    print(l, {k: [round(x[1] / 1e6, 2) for x in sorted(v)] for k, v in acc.items()})
PY
