"""The N > 1 bench path end to end on one GPU: bench.py under torchrun with two
ranks sharing cuda:0 (--share-gpu: peer transports only, RCCL refuses two ranks
on one device).  Checks the driver's contract on the line rank 0 prints — one
JSON line, the BASELINE metric, n_gpus, the weak-scaling value from its own
ms_per_step, a transport that was verified on this machine, no peer timeout —
not the numbers (a shared GPU measures nothing).  The 8-GPU run is the
driver's; this keeps the code path it takes exercised on every GPU run."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

pytestmark = pytest.mark.gpu


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_share_gpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--share-gpu", "--steps", "10", "--warmup", "2", "--no-extras",
           "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["metric"] == bench.METRIC and d["n_gpus"] == 2 and d["steps"] == 10 and d["scaling"] == "weak"
    world_bytes = 2 * bench.RANKS * bench.ELEMS * 2
    assert d["value"] == pytest.approx(world_bytes / (d["ms_per_step"] * 1e-3) / 1e9, rel=1e-3)
    x = d["xgmi"]
    transport = d["config"]["transport"]
    assert transport == x["headline_transport"]
    # the headline transport passed both independent checks on this machine
    v = x["transport_verified"][transport]
    assert v["verified"] is True and v["exact_sum"] is True and v["closed_form"] is True
    assert d["config"]["verified"] is True
    assert x["peer_timeout_in_timed_loop"] is False and x["peer_status"] & 1 == 0
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1
    assert x["timing"]["repetitions"] >= 3   # median of >= 3 K-step repetitions
    assert d["ms_per_step"] == pytest.approx(sorted(x["timing"]["ms_per_step_per_repetition"])[
        len(x["timing"]["ms_per_step_per_repetition"]) // 2], rel=1e-3)
    # the wall-clock budget (--deadline, default 420 s from the start of bench.py): every phase timed
    b = x["budget"]
    assert b["deadline_s"] == 420.0 and 0 < b["wall_s"] < b["deadline_s"]
    assert {"setup", "headline", "local_phases"} <= set(b["phase_s"]) and b["skipped_for_deadline"] == []
    assert any(k.startswith("verify:") for k in b["phase_s"]) and any(k.startswith("quick:") for k in b["phase_s"])


ONE_RANK_RCCL = r"""
import json, os, sys
sys.path.insert(0, sys.argv[1])
import torch, torch.distributed as dist
import bench
dist.init_process_group("gloo", rank=0, world_size=1)
torch.cuda.set_device(0)
probe = bench.link_probe(0, 1, "cuda:0")
comp = bench.rccl_allreduce_comparator(0, 1, "cuda:0", sizes=(("small_64kB", 64 << 10, 5), ("config4_1GiB", 1 << 30, 2)))
dist.destroy_process_group()
print(json.dumps({"probe": probe, "comp": comp}))
"""


def test_rccl_side_extras_run_over_torch_nccl_with_one_rank():
    """The two N > 1 extras that only run with an RCCL communicator and world > 1
    (link_probe, rccl_allreduce_comparator) have no --share-gpu rehearsal: RCCL
    refuses two ranks on one device.  Their code — torch's nccl group created from
    the gloo default group, the batched sendrecv, the exact-integer fill and check
    of a 1 GiB bf16 bucket on the device, the group's teardown — runs here on one
    rank, so the first multi-GPU node meets code that already ran on this chip."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    p = subprocess.run([sys.executable, "-c", ONE_RANK_RCCL, ROOT], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert d["probe"]["bytes"] == 128 << 20 and d["probe"]["reps"] == 5
    for name in ("small_64kB", "config4_1GiB"):
        c = d["comp"][name]
        assert c["verified_exact"] is True and c["ms"] > 0 and c["busbw_GBps"] == 0.0   # 2(p-1)/p = 0 at p = 1


def run_hung(phase: str, hard_s: int, how: str = "HANG"):
    env = dict(os.environ, ALLRED_BENCH_HARD_S=str(hard_s))
    env[f"ALLRED_BENCH_TEST_{how}_IN"] = phase
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--share-gpu", "--steps", "10", "--warmup", "2", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=hard_s + 120)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (p.stdout[-2000:], p.stderr[-3000:])
    return p, json.loads(lines[0])


def test_last_resort_watchdog_before_anything_is_measured():
    """A host-side hang before any number exists (here: in the peer comparator's
    verification; on a node, e.g. RCCL setup) ends at the last-resort watchdog with one
    line: value null, the phase it hung in, and a failing exit status."""
    p, d = run_hung("verify:peer_launches", 45)
    assert p.returncode != 0
    assert d["metric"] == bench.METRIC and d["value"] is None and d["n_gpus"] == 2
    assert "phase: verify:peer_launches" in d["error"] and d["xgmi"]["budget"]["phase_now"] == "verify:peer_launches"


def test_last_resort_watchdog_after_the_headline():
    """A hang after the headline (here: rank 0 entering cli_config3 while the others wait at
    the final barrier) still prints the measured line — the verified headline with the extras
    gathered so far and xgmi.watchdog — and every rank exits 0."""
    p, d = run_hung("cli_config3", 50)
    assert p.returncode == 0, p.stderr[-3000:]
    assert d["metric"] == bench.METRIC and d["value"] > 0 and d["config"]["verified"] is True
    x = d["xgmi"]
    assert "phase: cli_config3" in x["watchdog"] and x["budget"]["phase_now"] == "cli_config3"
    assert "headline" in x["budget"]["phase_s"] and "cli_config3" not in x


def test_an_error_before_anything_is_measured_still_prints_one_line():
    """An exception on rank 0 before any number exists (here: raised entering the headline
    phase) prints one line — value null, the error and the phase — and fails the run."""
    p, d = run_hung("headline", 120, how="RAISE")
    assert p.returncode != 0
    assert d["metric"] == bench.METRIC and d["value"] is None
    assert "test error in headline" in d["error"] and "(phase: headline)" in d["error"]
