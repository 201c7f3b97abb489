"""allred_run across G GPUs (ALLRED_GPUS / argv[10]) executed on hardware: the
same orchestration the 8-GPU node will run — G host threads, the two status
barriers, per-GPU H2D / D2H slices of the pinned host buckets, the timed
region, validation of every rank — with the exchange on the peer-window
transport (allred_peer_connect_all: the G threads' windows mapped into each
other) and every group on the one GPU of the box (ALLRED_SHARE_GPU=1).
RCCL refuses two ranks on one GPU, so this is the hardware rehearsal of the
multi-GPU program surface; the RCCL backend shares every line but the
exchange and the waits (csrc/multi.cpp).

Each case runs in a process of its own (the executable, or
tests/gpu_multi_child.py) with GPU_MAX_HW_QUEUES above G + 1 so that the G
threads' mutually waiting kernels never share a hardware queue; every peer
wait is bounded (a stall ends as ALLRED_ERR_TRANSPORT, not a hang).  The
timed region finishes the allreduce before the read-back (the reference's
RunProgram order): a D2H queued behind a waiting allreduce held a copy engine
another group's H2D was queued behind, and the groups deadlocked until the
4 s wait bound (profiles/r04_multi_share_trace.txt).
Reference: allred_BO_2D.cpp:7-29, allred_helper.cpp:205-220,
allred_helper.hpp:84-96."""
import os
import subprocess
import sys

import numpy as np
import pytest

import tenstorrentallreduce_amd as t
from multi_cases import BIN, argv_error0, expected, invocations

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _env(g, nodes):
    e = dict(os.environ)
    e.update({"ALLRED_TRANSPORT": "peer", "ALLRED_SHARE_GPU": "1", "ALLRED_GPUS": str(g),
              "GPU_MAX_HW_QUEUES": "16", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    e.pop("ALLRED_NODES", None)
    if nodes is not None:
        e["ALLRED_NODES"] = str(nodes)
    return e


GROUPS = [int(x) for x in os.environ.get("ALLRED_TEST_SHARE_GROUPS", "2,4,8").split(",")]
CASES = [(g, *inv) for g in GROUPS for inv in invocations(g)]


@pytest.mark.parametrize("g,name,variant,argv,nodes", CASES, ids=[f"g{c[0]}-{c[1]}" for c in CASES])
def test_cli_across_gpus_on_one_device(g, name, variant, argv, nodes):
    """The executable with ALLRED_GPUS=G: "All values match!" at ERROR 0, RNE
    ctor, every rank validated (strict exit code)."""
    env = _env(g, nodes)
    env.update({"ALLRED_CHECK_ALL": "1", "ALLRED_BF16_ROUND": "rne", "ALLRED_STRICT": "1", "ALLRED_REPORT": "1"})
    r = subprocess.run([os.path.join(t._lib.BIN_DIR, BIN[variant]), *argv_error0(argv, variant)],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)
    assert r.stdout.strip() == "All values match!", r.stdout
    assert '"mismatches": 0' in r.stderr


@pytest.mark.parametrize("g,name,variant,argv,nodes", CASES, ids=[f"g{c[0]}-{c[1]}" for c in CASES])
def test_across_gpus_bit_exact_vs_oracle_composition(tmp_path, g, name, variant, argv, nodes):
    """Arbitrary per-rank data through the G-thread orchestration on the GPU:
    every rank equals the oracle's composition of the plan bit for bit."""
    out = tmp_path / "out.npy"
    seed = 77 * g + len(name)
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_multi_child.py"), str(variant), str(g),
                        "-" if nodes is None else str(nodes), str(seed), str(out), "--", *argv],
                       capture_output=True, text=True, env=_env(g, nodes), timeout=180)
    assert r.returncode == 0, (r.stdout, r.stderr)
    data, got = np.load(out)
    env_nodes = os.environ.get("ALLRED_NODES")
    try:
        if nodes is None:
            os.environ.pop("ALLRED_NODES", None)
        else:
            os.environ["ALLRED_NODES"] = str(nodes)
        plan = t.multi_plan(["x", *argv], variant, gpus=g)
    finally:
        if env_nodes is None:
            os.environ.pop("ALLRED_NODES", None)
        else:
            os.environ["ALLRED_NODES"] = env_nodes
    want = expected(plan, data)
    bad = int((got != want).sum())
    assert bad == 0, f"{name} G={g}: {bad} elements differ"


@pytest.mark.parametrize("g,bad", [(2, 2), (4, 1), (4, 35)])
def test_failed_gpu_ends_every_thread_on_the_gpu(g, bad):
    """One group fails its timed allreduce (tune multi_fault 1..32) while the other
    groups' peer kernels wait for it, or its warm-up (33..64: every thread
    skips the timed region): their waits are bounded (4 s of
    s_memrealtime), every thread returns and the executable exits 1 with the
    transport error instead of hanging."""
    import time
    env = _env(g, 8)
    env["ALLRED_TUNE"] = f"multi_fault={bad}"
    t0 = time.monotonic()
    r = subprocess.run([os.path.join(t._lib.BIN_DIR, "allred_BO_2D"), "0", "1", "4", "13", "40", "32", "0", "1"],
                       capture_output=True, text=True, env=env, timeout=120)
    dt = time.monotonic() - t0
    assert r.returncode == 1, (r.stdout, r.stderr)
    assert "exchange callback failed" in r.stderr, r.stderr
    assert dt < 60, dt
