#!/usr/bin/env python3
"""Per-bounce durations of the wavefront launches in a rocprofv3 kernel trace: for the last
timed render, the extend / shade kernel of every bounce (us) and the gaps between them."""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    wf = [r for r in rows if "wf_extend" in r["Kernel_Name"] or "wf_shade" in r["Kernel_Name"]]
    # the stats pass and the timed renders: take the last 2*bounces launches
    ext = [i for i, r in enumerate(wf) if "wf_extend" in r["Kernel_Name"]]
    if not ext:
        raise SystemExit("no wavefront launches")
    # a render starts with bounce 0: extend launches whose predecessor is a shade of the last bounce
    starts = [i for i in ext if i == 0 or int(wf[i]["Start_Timestamp"]) - int(wf[i - 1]["End_Timestamp"]) > 50_000]
    last = wf[starts[-1]:]
    t0 = int(last[0]["Start_Timestamp"])
    tot_e = tot_s = 0
    prev_end = t0
    print(f"{'launch':<10}{'start_us':>10}{'dur_us':>10}{'gap_us':>8}")
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        kind = "extend" if "wf_extend" in r["Kernel_Name"] else "shade"
        if kind == "extend":
            tot_e += e - s
        else:
            tot_s += e - s
        print(f"{kind:<10}{(s - t0) / 1e3:>10.1f}{(e - s) / 1e3:>10.1f}{(s - prev_end) / 1e3:>8.1f}")
        prev_end = e
    print(f"extend total {tot_e / 1e3:.1f} us, shade total {tot_s / 1e3:.1f} us, span {(prev_end - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
