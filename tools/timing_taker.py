"""Timing sweep with the reference harness's shape (python/timing_taker.py:19-101)
and its analyzer statistics (python/profiler_results_analyzer.py:37-56).

Runs the MI355X executables with the reference's own invocation
  <bin> <swing> 1 8 13 <size> 32 0 <bo>
under ALLRED_PROFILE_LOG (the reference's TT_METAL_DEVICE_PROFILER=1: the
schedule form stamps every unit on the device and the library writes each
rank's ALL_RED_LOOP zone in the profile_log_device.csv layout), runs the
reference's timing-distribution analysis on it (normalized start / end per
core, tools/profile_analyzer.py normalized()), and appends the reference's
row: mode, swing_algo, data_size, run_num, then the 64 cores' normalized
starts and the 64 normalized ends (python/timing_taker.py:19-23, 79-101;
100 MHz ticks), then device_ns, e2e_ns, mismatches.  `--summary` prints the
analyzer's min / Q1 / mean / median / Q3 / max of the per-core zone lengths
(profiler_results_analyzer.py:37-56) per (mode, algo, size).

  python tools/timing_taker.py [--runs 20] [--exec steps|fused] [--out results.csv] [--summary]
"""
import argparse
import csv
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODES = ["allred_BO_2D", "allred_LO_2D", "allred_mem_2D"]           # timing_taker.py:11
SWING_LO_BO = [0, 1]                                                # :13
SWING_MEM = [1]                                                     # :14
SIZES_LO = [1, 2, 4, 8, 16, 32, 64, 128, 192, 256, 320]            # :15
SIZES_BO_MEM = [1, 2, 3, 4, 5]                                      # :16
RANGE_X = [1, 2, 3, 4, 6, 7, 8, 9]                                  # :17
RANGE_Y = [1, 2, 3, 4, 5, 7, 8, 9]                                  # :18


def plan():
    for mode in MODES:
        if mode == "allred_BO_2D":      # :34-38
            yield mode, "allred_BO_2D", SWING_LO_BO, SIZES_BO_MEM, "1"
        elif mode == "allred_LO_2D":    # :39-43 (LO through the BO binary, arg 8 = 0)
            yield mode, "allred_BO_2D", SWING_LO_BO, SIZES_LO, "0"
        else:
            yield mode, "allred_mem_2D", SWING_MEM, SIZES_BO_MEM, None


def header():
    return (["mode", "swing_algo", "data_size", "run_num"] + [f"{x}{y}_start" for y in RANGE_Y for x in RANGE_X] +
            [f"{x}{y}_end" for y in RANGE_Y for x in RANGE_X] + ["device_ns", "e2e_ns", "mismatches"])


def row_from_log(mode, swing, size, run, log, rep) -> list:
    """The reference's CSV row (python/timing_taker.py:83-101): the 64 cores'
    normalized starts, then their ends ("N/A" for a core without a zone)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from profile_analyzer import normalized
    core = normalized(log)
    starts = [core.get((x, y), ("N/A", "N/A"))[0] for y in RANGE_Y for x in RANGE_X]
    ends = [core.get((x, y), ("N/A", "N/A"))[1] for y in RANGE_Y for x in RANGE_X]
    return [mode, swing, size, run, *starts, *ends, round(rep["device_s"] * 1e9), round(rep["e2e_s"] * 1e9),
            rep["mismatches"]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--exec", default="steps", choices=["steps", "fused"],
                    help="steps: the schedule form (per-rank device stamps); fused: one interval for all ranks")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "profiler_results.csv"))
    ap.add_argument("--summary", action="store_true")
    args = ap.parse_args()
    import tenstorrentallreduce_amd as t
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    log = os.path.join(os.path.dirname(args.out), "profile_log_device.csv")
    rows = []
    for run in range(args.runs):
        print(f"[timing_taker] run {run + 1}/{args.runs}", file=sys.stderr, flush=True)   # progress (long sweeps)
        for mode, binary, algos, sizes, bo in plan():
            for swing in algos:
                for size in sizes:
                    argv = [str(swing), "1", "8", "13", str(size), "32"] + (["0", bo] if bo is not None else [])
                    # device_ns = the allreduce on device-resident buckets (the reference's
                    # ALL_RED_LOOP zone), so the host buckets move by DMA before and after it
                    p = t.run_cli(binary, argv, env={"ALLRED_REPORT": "1", "ALLRED_EXEC": args.exec,
                                                     "ALLRED_E2E": "dma", "ALLRED_PROFILE_LOG": log})
                    rep = json.loads(p.stderr.strip().splitlines()[-1])
                    rows.append(row_from_log(mode, swing, size, run, log, rep))
    with open(args.out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header())
        w.writerows(rows)
    if args.summary:
        groups = {}
        for row in rows:
            mode, swing, size = row[:3]
            zones = [e - s for s, e in zip(row[4:68], row[68:132]) if s != "N/A" and e != "N/A"]
            groups.setdefault((mode, swing, size), []).extend(z * 10 for z in zones)   # ticks -> ns
        print("mode,swing_algo,data_size,min_ns,q1_ns,mean_ns,median_ns,q3_ns,max_ns   (per-core ALL_RED_LOOP zones)")
        for (mode, swing, size), v in groups.items():
            a = np.array(v, dtype=float)
            print(f"{mode},{swing},{size},{a.min():.0f},{np.percentile(a, 25):.0f},{a.mean():.0f},"
                  f"{np.median(a):.0f},{np.percentile(a, 75):.0f},{a.max():.0f}")


if __name__ == "__main__":
    main()
