"""bench.py's contract without a GPU: the metric is BASELINE.json's, the N = 1
workload is BASELINE config 2 (8x8 Swing BO, 64 ranks x 655,360 B), and the
argument surface the driver uses exists with the documented defaults."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_metric_is_baselines():
    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert bench.METRIC == baseline["metric"]


def test_workload_is_config2():
    assert (bench.SIDE, bench.RANKS, bench.TILES) == (8, 64, 5)
    assert bench.ELEMS * 2 == 655360                     # 655,360 B per rank
    assert 2 * bench.RANKS * bench.ELEMS * 2 == 83886080  # algorithmic HBM bytes per launch


def test_gpu_grids_map_onto_the_reference_2d_functions():
    # 2 GPUs (2,2), 4 GPUs (2,4), 8 GPUs (4,8)
    assert bench.GRIDS[2] == (2, 2) and bench.GRIDS[4] == (2, 4) and bench.GRIDS[8] == (4, 8)


def test_n_gt_1_budget_skips_extras_before_the_deadline(monkeypatch):
    """The N > 1 line's wall-clock budget (verdict r05 item 2): a phase starts only
    while the time left covers max(60 s, 2 x the longest phase so far); skipped
    phases are listed, every phase's seconds are reported, and the default
    deadline sits well under the driver's 600 s lease."""
    now = [1000.0]
    monkeypatch.setattr(bench.time, "perf_counter", lambda: now[0])
    b = bench.Budget(420.0, t0=1000.0)
    with b.phase("setup"):
        now[0] += 30.0
    assert b.allows("arm:a", agree=False)            # 390 s left > max(60, 60)
    with b.phase("arm:a"):
        now[0] += 100.0                               # a long arm: 100 s
    assert b.allows("arm:b", agree=False)            # 290 s left > 200
    with b.phase("arm:b"):
        now[0] += 90.0
    assert not b.allows("arm:c", agree=False)        # 200 s left: not more than 2 x 100
    now[0] += 100.0
    assert not b.allows("cpu_baseline", agree=False)
    r = b.report()
    assert r["phase_s"] == {"setup": 30.0, "arm:a": 100.0, "arm:b": 90.0}
    assert r["skipped_for_deadline"] == ["arm:c", "cpu_baseline"]
    assert r["wall_s"] == 320.0 and r["deadline_s"] == 420.0
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'ap.add_argument("--deadline", type=float, default=420.0' in src   # < the driver's 600 s


def test_last_resort_watchdog_line(monkeypatch):
    """main()'s last-resort watchdog for the N > 1 run (a host-side hang no phase watchdog
    covers): with nothing measured it prints a line with value null, the metric and the phase
    it hung in; once a line was measured (the RCCL fallback, then the headline) it prints that
    line with xgmi.watchdog."""
    import argparse
    args = argparse.Namespace(steps=20, warmup=5)
    now = [0.0]
    monkeypatch.setattr(bench.time, "perf_counter", lambda: now[0])
    b = bench.Budget(420.0, t0=0.0)
    monkeypatch.setattr(bench, "BUDGET", [b])
    monkeypatch.setattr(bench, "BEST_LINE", [None])
    with b.phase("setup"):
        now[0] += 3.0
    cm = b.phase("verify:rccl")
    cm.__enter__()                                   # hangs in here
    now[0] += 537.0
    ln = bench.watchdog_line(args, 8, "hung")
    assert ln["metric"] == bench.METRIC and ln["value"] is None and ln["n_gpus"] == 8
    assert ln["error"] == "hung (phase: verify:rccl)" and ln["xgmi"]["budget"]["phase_now"] == "verify:rccl"
    assert ln["xgmi"]["budget"]["phase_s"] == {"setup": 3.0}
    bench.BEST_LINE[0] = lambda: {"metric": bench.METRIC, "value": 123.0, "xgmi": {"headline_transport": "rccl"}}
    ln = bench.watchdog_line(args, 8, "hung")
    assert ln["value"] == 123.0 and "phase: verify:rccl" in ln["xgmi"]["watchdog"]

    def broken():
        raise RuntimeError("boom")
    bench.BEST_LINE[0] = broken                       # a line that cannot be rebuilt: still a line
    ln = bench.watchdog_line(args, 8, "hung")
    assert ln["value"] is None and "boom" in ln["error"]
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'os.environ.get("ALLRED_BENCH_HARD_S", args.deadline + 120.0)' in src   # 540 s < the 600 s lease
