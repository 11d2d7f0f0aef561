#!/usr/bin/env python3
"""Record one rocprofv3 profile of a bench.py command into profiles/pmc.json.

usage: pmc_record.py TRACE_DIR PMC_DIR [PMC_DIR ...] -- [bench.py args]
TRACE_DIR holds the --kernel-trace --stats pass (kernel_stats.csv), each PMC_DIR one --pmc
pass of the SAME bench command.  The entry is keyed like bench.py's roofline lookup
(workload_key) and stamped with bench.kernel_source_hash(), so a later kernel change marks it
stale instead of silently mis-pricing the new build.  HBM bytes per launch =
(2 * FETCH_SIZE + WRITE_SIZE) KiB: on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B stores.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def render_kernel(names):
    """The timed render launch: KernelEntry's step entry point specialised for a launch kind (its
    last template argument, kMode, 1 fused or 2 per-frame; the stats variant that the count pass
    runs is the generic body, kMode 0), else -- other schedules -- the entry point whose first
    template argument, kStats, is false."""
    c = [k for k in names if "kernel_entry" in k and re.search(r", [12]>", k)]
    if not c:
        c = [k for k in names if "kernel_entry" in k and "<false" in k]
    return c[0] if c else None


def main():
    sep = sys.argv.index("--")
    dirs, bench_args = sys.argv[1:sep], sys.argv[sep + 1:]
    trace_dir, pmc_dirs = dirs[0], dirs[1:]
    sys.argv = ["bench.py"] + bench_args
    import bench
    args = bench.parse()
    frames_per_launch = args.frames if (args.launch == "fused" and args.sched in ("step", "wavefront")) else 1
    key = bench.workload_key(args, int(os.environ.get("WORLD_SIZE", "1")), frames_per_launch)

    acc = defaultdict(lambda: defaultdict(list))
    for d in pmc_dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    k = render_kernel(acc)
    if k is None:
        raise SystemExit("no render kernel in the PMC passes")
    e = {c: sum(v) / len(v) for c, v in acc[k].items()}
    e["kernel"] = k
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
        e["hbm_bytes_per_launch"] = int((2.0 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024.0)
    for f in glob.glob(os.path.join(trace_dir, "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Name"] == k:
                e["kernel_ms"] = float(row["AverageNs"]) / 1e6
    # the fused launches' accumulation (accum_frames*, on its own stream beside the next render):
    # its VALU shares the render's SIMDs, so the bench line prices it too (roofline.accum_*)
    acc_k = [n for n in acc if "accum_frames" in n]
    if acc_k:
        a = {c: sum(v) / len(v) for c, v in acc[acc_k[0]].items()}
        e["accum"] = {"kernel": acc_k[0], **{c: a[c] for c in ("SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_SALU",
                                                            "SQ_WAVE_CYCLES") if c in a}}
    e["source_hash"] = bench.kernel_source_hash()
    e["command"] = "python bench.py " + " ".join(bench_args)
    path = os.path.join(REPO, "profiles", "pmc.json")
    db = json.load(open(path)) if os.path.exists(path) else {}
    db[key] = e
    json.dump(db, open(path, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(e, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
