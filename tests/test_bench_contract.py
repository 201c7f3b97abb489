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
