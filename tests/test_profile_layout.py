"""The profiling CSV contract without a GPU: the
profile_log_device.csv layout the engine (allred_run, ALLRED_PROFILE_LOG) and
the CPU loopback baseline (ORACLE_PROFILE_LOG) both write, read by the
reference's analyses (python/profiler_results_analyzer*.py, restated in
tools/profile_analyzer.py) into the reference's timing_taker row: 64 cores'
normalized starts, then their normalized ends (python/timing_taker.py:19-23, 79-101)."""
import os
import sys

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from profile_analyzer import analyze, normalized  # noqa: E402
import timing_taker  # noqa: E402


def test_loopback_log_to_reference_row(tmp_path):
    log = str(tmp_path / "profile_log_device.csv")
    out = oracle.loopback("bo", [1, 1, 8, 13, 1, 32, 0, 0], reps=2, timeout=120, profile_log=log)
    assert out["mismatches"] == 0
    first = open(log).readline()
    assert first.startswith("ARCH:") and "CHIP_FREQ[MHz]" in first
    core = normalized(log)
    # the reference's 8x8 grid sits on these Wormhole worker cores (timing_taker.py:17-18)
    assert set(core) == {(x, y) for x in timing_taker.RANGE_X for y in timing_taker.RANGE_Y}
    assert min(s for s, _ in core.values()) == 0
    assert all(e > s for s, e in core.values())
    stats = analyze(log)
    assert stats["cores"] == 64 and stats["min"] > 0
    row = timing_taker.row_from_log("allred_LO_2D", 1, 1, 0, log,
                                    {"device_s": 1e-6, "e2e_s": 2e-6, "mismatches": 0})
    hdr = timing_taker.header()
    assert len(row) == len(hdr) == 4 + 64 + 64 + 3
    assert hdr[4] == "11_start" and hdr[4 + 64] == "11_end" and hdr[4 + 63] == "99_start"
    assert "N/A" not in row


def test_missing_core_is_na(tmp_path):
    log = str(tmp_path / "p.csv")
    out = oracle.loopback("bo", [0, 1, 2, -1, 1, 32, 0, 0], reps=1, timeout=60, profile_log=log)   # 2x2: 4 cores
    assert out["mismatches"] == 0
    row = timing_taker.row_from_log("allred_LO_2D", 0, 1, 0, log, {"device_s": 0, "e2e_s": 0, "mismatches": 0})
    starts = row[4:68]
    assert sum(1 for v in starts if v != "N/A") == 4
