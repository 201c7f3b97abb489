#!/usr/bin/env python3
"""Per-core ALL_RED_LOOP statistics of a tt-metal-layout profile log — the
computation of the reference's python/profiler_results_analyzer.py:5-56 (for
every core, the latest ZONE_START and ZONE_END over its RISC processors;
execution time = latest end - latest start; min / Q1 / mean / median / Q3 /
max over cores, with the min and max cores named).

Input: a CSV in the layout of profile_log_device.csv — the MI355X engine's
(ALLRED_PROFILE_LOG, allred_run: 100 MHz s_memrealtime ticks) or the CPU
loopback baseline's (ORACLE_PROFILE_LOG, oracle/allred_oracle_cli.c: ns).
normalized() is the timing-distribution analysis
(python/profiler_results_analyzer_timing_distributions.py:5-48).
Usage: python tools/profile_analyzer.py <csv>
"""
from __future__ import annotations

import json
import sys

import numpy as np
import pandas as pd


def analyze(csv_file: str, run_id: int | None = None) -> dict:
    """run_id: only that run's zones (the loopback log holds every rep)."""
    df = pd.read_csv(csv_file, skiprows=1)
    loop = df[df["  zone name"] == "ALL_RED_LOOP"]
    if run_id is not None:
        loop = loop[loop[" run ID"] == run_id]
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


def normalized(csv_file: str) -> dict:
    """python/profiler_results_analyzer_timing_distributions.py:5-48: per core
    (x, y), the latest ZONE_START and latest ZONE_END over its RISCs, both minus
    the earliest start of all cores.  {(x, y): (normalized_start, normalized_end)}"""
    df = pd.read_csv(csv_file, skiprows=1)
    loop = df[df["  zone name"] == "ALL_RED_LOOP"]
    latest: dict = {}
    for (x, y, proc, phase), g in loop.groupby([" core_x", " core_y", " RISC processor type", " type"]):
        latest.setdefault((int(x), int(y)), {}).setdefault(phase, {})[proc] = int(g[" time[cycles since reset]"].max())
    core = {k: (max(v["ZONE_START"].values()), max(v["ZONE_END"].values()))
            for k, v in latest.items() if "ZONE_START" in v and "ZONE_END" in v}
    if not core:
        return {}
    t0 = min(s for s, _ in core.values())
    return {k: (s - t0, e - t0) for k, (s, e) in core.items()}


if __name__ == "__main__":
    r = analyze(sys.argv[1])
    print(f"Min: {r['min']} (Core {r['min_core'][0]},{r['min_core'][1]})")
    print(f"Lower Quartile: {r['q1']}")
    print(f"Mean: {r['mean']}")
    print(f"Median: {r['median']}")
    print(f"Upper Quartile: {r['q3']}")
    print(f"Max: {r['max']} (Core {r['max_core'][0]},{r['max_core'][1]})")
    print(json.dumps(r))
