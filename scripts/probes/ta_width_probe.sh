# TA cost of a divergent load by width and addressing form (scripts/probes/ta_width_probe.hip):
# ns per wave-visit from HIP events at 64 / 40 / 16 active lanes, then TA busy cycles per dispatch
set -o pipefail
export TMPDIR=/tmp
for n in 64 40 16; do
  timeout -k 10 60 scripts/probes/ta_width_probe $n || exit 1
done
timeout -k 10 60 rocprofv3 --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ta_width -o run -- scripts/probes/ta_width_probe 64 > /dev/null 2>&1 || exit 1
python3 - gpurun_out/ta_width <<'PY'
import csv, glob, sys
from collections import defaultdict
rows = defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[int(r["Dispatch_Id"])]["name"] = r["Kernel_Name"][:22]
visits = 256 * 8 * 4 * 2000
for d in sorted(rows):
    r = rows[d]
    print(f"dispatch {d} {r['name']}: TA busy {r.get('TA_TA_BUSY_sum', 0):.3e}, TA cycles per wave-visit per CU-TA {r.get('TA_TA_BUSY_sum', 0) / visits:.2f}")
PY
