#!/usr/bin/env python3
"""Per-launch time of the fused render from a rocprofv3 kernel trace: consecutive renders overlap on
two streams, so a launch's span (start -> end) includes time shared with its neighbour; the
interval between consecutive render ends is what each launch costs (bench.py's launch_ms).
usage: trace_period.py run_kernel_trace.csv [kernel-substring]"""
import csv
import sys


def main(path, sub="kernel_entry_step_shipped_lds<false"):
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["End_Timestamp"]))
    print(f"{'launch':>6} {'span_ms':>9} {'end_to_end_ms':>14}   ({rows[0]['Kernel_Name'] if rows else sub})")
    periods = []
    for i, r in enumerate(rows):
        span = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        per = (int(r["End_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e6 if i else None
        if per is not None and i > 1:
            periods.append(per)
        print(f"{i:>6} {span:>9.3f} {per if per is None else round(per, 3)!s:>14}")
    if periods:
        print(f"mean end-to-end interval of the timed launches: {sum(periods) / len(periods):.3f} ms")


if __name__ == "__main__":
    main(*sys.argv[1:])
