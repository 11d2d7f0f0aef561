# round-5 A/B session 4: radiance staged in LDS on the fused HBM/L2 octant walk (main) against the same
# source without it (nostage) and HEAD before it (headref): fused-frame parity tests, bunny and Cornell
# benches, bunny write counters
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_frames.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab4_tests.txt 2>&1 || { tail -30 gpurun_out/ab4_tests.txt; exit 1; }
tail -2 gpurun_out/ab4_tests.txt
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 --no-drop-in --scene bunny || exit 1
bash scripts/ab_quick.sh 1 --no-drop-in || exit 1
for l in main nostage; do
  if [ $l = main ]; then unset RT_HIP_LIB; else export RT_HIP_LIB=mini-opencl-raytracer_amd/lib/variants/librt_hip_$l.so; fi
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/wr4_$l -o run -- python bench.py --scene bunny --steps 1 --warmup 0 --no-cpu-baseline --no-drop-in > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for l in ("main", "nostage"):
    acc = defaultdict(list)
    for f in glob.glob(f'gpurun_out/wr4_{l}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'goct' in r['Kernel_Name']:
                acc[r['Counter_Name']].append((int(r['Dispatch_Id']), float(r['Counter_Value'])))
    print(l, {k: [round(x[1] / 1e6, 3) for x in sorted(v)] for k, v in acc.items()})
PY
