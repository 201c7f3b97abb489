#!/usr/bin/env python3
"""Per-core ALL_RED_LOOP statistics of a tt-metal-layout profile log — the
computation of the reference's python/profiler_results_analyzer.py:5-56 (for
every core, the latest ZONE_START and ZONE_END over its RISC processors;
execution time = latest end - latest start; min / Q1 / mean / median / Q3 /
max over cores, with the min and max cores named).

Input: the CSV the CPU loopback baseline writes under ORACLE_PROFILE_LOG
(oracle/allred_oracle_cli.c), same columns and metadata line as
profile_log_device.csv.  Usage: python tools/profile_analyzer.py <csv>
"""
from __future__ import annotations

import json
import sys

import numpy as np
import pandas as pd


def analyze(csv_file: str) -> dict:
    df = pd.read_csv(csv_file, skiprows=1)
    loop = df[df["  zone name"] == "ALL_RED_LOOP"]
    latest: dict = {}
    for (x, y, proc, phase), g in loop.groupby([" core_x", " core_y", " RISC processor type", " type"]):
        t = g[" time[cycles since reset]"].max()
        latest.setdefault((x, y), {}).setdefault(phase, {})[proc] = t
    times = []
    for (x, y), ph in latest.items():
        if "ZONE_START" in ph and "ZONE_END" in ph:
            times.append((max(ph["ZONE_END"].values()) - max(ph["ZONE_START"].values()), x, y))
    v = np.array([t for t, _, _ in times], dtype=np.float64)
    lo = min(times)
    hi = max(times)
    return {"cores": len(times), "min": float(v.min()), "min_core": [int(lo[1]), int(lo[2])],
            "q1": float(np.percentile(v, 25)), "mean": float(v.mean()), "median": float(np.median(v)),
            "q3": float(np.percentile(v, 75)), "max": float(v.max()), "max_core": [int(hi[1]), int(hi[2])]}


if __name__ == "__main__":
    r = analyze(sys.argv[1])
    print(f"Min: {r['min']} (Core {r['min_core'][0]},{r['min_core'][1]})")
    print(f"Lower Quartile: {r['q1']}")
    print(f"Mean: {r['mean']}")
    print(f"Median: {r['median']}")
    print(f"Upper Quartile: {r['q3']}")
    print(f"Max: {r['max']} (Core {r['max_core'][0]},{r['max_core'][1]})")
    print(json.dumps(r))
