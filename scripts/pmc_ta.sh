# texture-address / data pipe occupancy of the render launch (is a divergent-gather walk bound by
# the vector memory pipe?): two PMC passes of bench.py, args as scripts/profile.sh
set -u
NAME=$1; shift
OUT=gpurun_out/pmc_ta_$NAME; mkdir -p $OUT; export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o run -- $B > $OUT/a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o run -- $B > $OUT/b.log 2>&1 || exit 1
python3 - $OUT <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    if "kernel_entry" in k and "<false" in k:
        print(k[:60], {n: sum(v) / len(v) for n, v in c.items()})
PY
