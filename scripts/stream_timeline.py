#!/usr/bin/env python3
"""Dispatch timeline of a rocprofv3 kernel trace (plus its memory-copy trace, when present): every
kernel and copy with its hardware queue / stream ids and start / end relative to the first
render, so one can read which launches waited for which (e.g. a fused render that starts only
when the previous step's gather transfer ends).
usage: stream_timeline.py TRACE_DIR_OR_CSV [--last N]"""
import csv
import glob
import os
import sys


def short(name):
    n = name.split("(")[0]
    for key, tag in (("kernel_entry_step", "RENDER"), ("accum_frames", "ACCUM"), ("accum", "ACCUM"),
                     ("nccl", "RCCL"), ("rccl", "RCCL"), ("Copy", "COPY"), ("copy", "COPY"), ("Fill", "FILL")):
        if key in n:
            return f"{tag:6s} {n[:60]}"
    return f"{'other':6s} {n[:60]}"


def load(path):
    files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
        for m in glob.glob(os.path.join(os.path.dirname(f), "*memory_copy_trace.csv")):
            for r in csv.DictReader(open(m)):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             f"MEMCPY {r.get('Direction', '')}", "sdma", r.get("Stream_Id", "?")))
    rows.sort()
    return rows


def main(argv):
    path = argv[0]
    last = int(argv[argv.index("--last") + 1]) if "--last" in argv else 80
    rows = load(path)
    renders = [r for r in rows if r[2].startswith("RENDER")]
    t0 = renders[0][0] if renders else rows[0][0]
    print(f"{'start_ms':>9} {'end_ms':>9} {'dur_ms':>7} {'queue':>6} {'stream':>6}  kernel")
    for s, e, n, q, st in rows[-last:]:
        print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:7.3f} {q:>6} {st:>6}  {n}")
    # overlap of consecutive renders: how long render k+1 ran before render k ended
    ov = [(renders[i - 1][1] - renders[i][0]) / 1e6 for i in range(1, len(renders))]
    if ov:
        print("render k+1 start before render k end (ms; negative = a gap):",
              " ".join(f"{x:.3f}" for x in ov[-12:]))


if __name__ == "__main__":
    main(sys.argv[1:])
