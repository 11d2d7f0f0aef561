# TA cycles per divergent 16-B load wave-instruction vs active lanes (scripts/probes/ta_probe.hip)
set -o pipefail
export TMPDIR=/tmp
for n in 64 32 16 8; do
  timeout -k 10 60 scripts/probes/ta_probe $n || exit 1
  timeout -k 10 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ta_probe_$n -o run -- scripts/probes/ta_probe $n > /dev/null 2>&1 || exit 1
  python3 - gpurun_out/ta_probe_$n $n <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
ta, wf = sum(acc["TA_TA_BUSY_sum"]) / len(acc["TA_TA_BUSY_sum"]), sum(acc["TA_FLAT_READ_WAVEFRONTS_sum"]) / len(acc["TA_FLAT_READ_WAVEFRONTS_sum"])
print(f"active {sys.argv[2]}: TA busy {ta:.3e}, flat read wavefronts {wf:.3e}, TA cycles per wave-load {ta / wf:.2f}")
PY
done
