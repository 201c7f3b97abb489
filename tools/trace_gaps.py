#!/usr/bin/env python3
"""Back-to-back runs of one kernel in a rocprofv3 kernel trace: for every run of
consecutive dispatches of the kernel (no other kernel in between on the agent),
the dispatches, the mean kernel duration, the mean idle gap between one
dispatch's end and the next one's start, and the run's span per dispatch (what
a pair of HIP events around the run measures).  Tells a slow kernel from a
host-bound launch sequence (gaps) in a bench's timed region.

  python tools/trace_gaps.py <run_kernel_trace.csv> <kernel-substring> [min_run]"""
import csv
import statistics
import sys


def runs(path, sub, min_run=5):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out, cur = [], []
    for r in rows:
        if sub in r["Kernel_Name"]:
            cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            continue
        if len(cur) >= min_run:
            out.append(cur)
        cur = []
    if len(cur) >= min_run:
        out.append(cur)
    res = []
    for c in out:
        dur = [e - s for s, e in c]
        gaps = [c[i + 1][0] - c[i][1] for i in range(len(c) - 1)]
        res.append({"dispatches": len(c), "kernel_us": round(statistics.mean(dur) / 1e3, 3),
                    "gap_us": round(statistics.mean(gaps) / 1e3, 3) if gaps else 0.0,
                    "first_gap_us": round(gaps[0] / 1e3, 3) if gaps else 0.0,
                    "span_us_per_dispatch": round((c[-1][1] - c[0][0]) / len(c) / 1e3, 3)})
    return res


if __name__ == "__main__":
    for r in runs(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 5):
        print(r)
