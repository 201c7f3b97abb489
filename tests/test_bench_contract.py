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
