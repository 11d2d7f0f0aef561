#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per kernel over all of its dispatches, plus the trace's total
duration per kernel.  usage: pmc_sum.py DIR [--all]  (DIR from scripts/profile.sh or
scripts/pmc_variants.sh; --all: also kernels without SQ_INSTS_VALU)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, show_all=False):
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(d, "p_*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            n[k][row["Counter_Name"]] += 1
    dur = defaultdict(float)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            dur[row["Kernel_Name"]] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
    for k, cs in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0)):
        if cs.get("SQ_INSTS_VALU", 0) < 1e6 and not show_all:
            continue
        print(f"{k[:100]}  dispatches {max(n[k].values())}  trace ms {dur.get(k, 0):.3f}")
        v = cs.get("SQ_INSTS_VALU", 0)
        if v:
            print(f"   lane_util {cs.get('SQ_THREAD_CYCLES_VALU', 0) / 64 / v:.3f}   "
                  f"valu_frac {v / (1024 * 1.2e9 * dur.get(k, 1e9) * 1e-3):.3f}   "
                  f"lds_conflict/active_lds {cs.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, cs.get('SQ_ACTIVE_INST_LDS', 1)):.2f}   "
                  f"wait_inst_any/wave_cycles {cs.get('SQ_WAIT_INST_ANY', 0) / max(1, cs.get('SQ_WAVE_CYCLES', 1)):.2f}   "
                  f"hbm GB {(2 * cs.get('FETCH_SIZE', 0) + cs.get('WRITE_SIZE', 0)) * 1024 / 1e9:.3f}")
        for c, x in sorted(cs.items()):
            print(f"   {c:28s} {x:18.1f}")


if __name__ == "__main__":
    main(sys.argv[1], "--all" in sys.argv[2:])
