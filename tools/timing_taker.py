"""Timing sweep with the reference harness's shape (python/timing_taker.py:19-101)
and its analyzer statistics (python/profiler_results_analyzer.py:37-56).

Runs the MI355X executables with the reference's own invocation
  <bin> <swing> 1 8 13 <size> 32 0 <bo>
for the reference's modes, algorithms, sizes and run count, and writes one CSV
row per run: mode, swing_algo, data_size, run_num, device_ns, e2e_ns,
mismatches (the reference's row carries 64 per-core Tracy start/end stamps of
the ALL_RED_LOOP zone; on MI355X the allreduce is one device-side interval per
run, timed with HIP events — `ALLRED_REPORT=1`).  `--summary` prints the
analyzer's min / Q1 / mean / median / Q3 / max per (mode, algo, size).

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


def plan():
    for mode in MODES:
        if mode == "allred_BO_2D":      # :34-38
            yield mode, "allred_BO_2D", SWING_LO_BO, SIZES_BO_MEM, "1"
        elif mode == "allred_LO_2D":    # :39-43 (LO through the BO binary, arg 8 = 0)
            yield mode, "allred_BO_2D", SWING_LO_BO, SIZES_LO, "0"
        else:
            yield mode, "allred_mem_2D", SWING_MEM, SIZES_BO_MEM, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--exec", default="steps", choices=["steps", "fused"])
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "profiler_results.csv"))
    ap.add_argument("--summary", action="store_true")
    args = ap.parse_args()
    import tenstorrentallreduce_amd as t
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
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
                                                     "ALLRED_E2E": "dma"})
                    rep = json.loads(p.stderr.strip().splitlines()[-1])
                    rows.append([mode, swing, size, run, round(rep["device_s"] * 1e9), round(rep["e2e_s"] * 1e9),
                                 rep["mismatches"]])
    with open(args.out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["mode", "swing_algo", "data_size", "run_num", "device_ns", "e2e_ns", "mismatches"])
        w.writerows(rows)
    if args.summary:
        groups = {}
        for mode, swing, size, run, dev, e2e, bad in rows:
            groups.setdefault((mode, swing, size), []).append(dev)
        print("mode,swing_algo,data_size,min_ns,q1_ns,mean_ns,median_ns,q3_ns,max_ns")
        for (mode, swing, size), v in groups.items():
            a = np.array(v, dtype=float)
            print(f"{mode},{swing},{size},{a.min():.0f},{np.percentile(a, 25):.0f},{a.mean():.0f},"
                  f"{np.median(a):.0f},{np.percentile(a, 75):.0f},{a.max():.0f}")


if __name__ == "__main__":
    main()
