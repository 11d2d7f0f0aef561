#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).

usage: pmc_summary.py OUT.json DIR [DIR ...]   (each DIR holds a *counter_collection.csv)
Writes {kernel: {counter: mean_per_dispatch, ..., "dispatches": n}} to OUT.json and prints it.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[2:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"]
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k]["dispatches"] = max(len(v) for v in cs.values())
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, cs in res.items():
        if "kernel_entry" not in k:
            continue
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {v:16.1f}")


if __name__ == "__main__":
    main()
