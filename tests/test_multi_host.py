"""allred_run across G GPUs (ALLRED_GPUS / argv[10]) on CPU: the plan
(allred_multi_plan_build, no HIP call) and the whole orchestration — G
threads, barriers and status agreement, per-GPU input / output slices,
validation — on the host-twin backend (ALLRED_TRANSPORT=host: host memory,
allred_dist_allreduce_host with an in-memory exchange).  The GPU backends run
the same orchestration code (csrc/multi.cpp); only the memory, the exchange and
the waits differ.

For every INTEGRATION.md §1 invocation at G = 2, 4, 8:
- the executable prints "All values match!" at ERROR 0 under the RNE
  bfloat16 ctor with every rank validated (ALLRED_CHECK_ALL, ALLRED_STRICT);
- on arbitrary per-rank data the result equals the oracle's composition of
  the plan bit for bit (tests/multi_cases.py).
Reference: allred_BO_2D.cpp:7-29, allred_helper.cpp:205-220 (argv),
allred_helper.cpp:18-120 (the check), allred_helper.hpp:84-96 (RunProgram)."""
import os

import numpy as np
import pytest

import tenstorrentallreduce_amd as t
from multi_cases import BIN, argv_error0, expected, invocations, random_inputs


def _env(monkeypatch, nodes):
    if nodes is None:
        monkeypatch.delenv("ALLRED_NODES", raising=False)
    else:
        monkeypatch.setenv("ALLRED_NODES", str(nodes))


def test_plan_config3_flat_across_8_gpus(monkeypatch):
    """BASELINE config 3 (4x2 RecDub BO, one rank per GPU): the reference's own grid over the GPUs."""
    _env(monkeypatch, 8)
    p = t.multi_plan(["x", "0", "1", "4", "13", "40", "32", "0", "1"], t.BO, gpus=8)
    assert (p.gpus, p.local_ranks, p.total_nodes, p.mode, p.variant) == (8, 1, 8, t.MULTI_FLAT, t.BO)
    assert (p.desc.algo, p.desc.side_length, p.desc.total_nodes, p.desc.local_ranks) == (t.RECDUB, 4, 8, 1)
    assert p.elems == 40 * 8 * 1024 and p.validated_mask == 0xFF   # every GPU's first (= only) rank


@pytest.mark.parametrize("g,local_side", [(1, 8), (2, 8), (4, 4), (8, 4), (16, 2), (32, 2), (64, 1)])
def test_plan_64_ranks_hierarchical(monkeypatch, g, local_side):
    """64 ranks over G GPUs: L = 64/G consecutive ranks per GPU; their sub-grid is
    L/8 rows of the reference's 8-wide grid when that is a schedule."""
    _env(monkeypatch, None)
    p = t.multi_plan(["x", "1", "1", "8", "13", "5", "32", "0", "1"], t.BO, gpus=g)
    L = 64 // g
    assert (p.gpus, p.local_ranks) == (g, L)
    gside = {1: 1, 2: 2, 4: 2, 8: 4, 16: 4}.get(g, 8)
    if L == 1:
        assert p.mode == t.MULTI_FLAT and (p.desc.side_length, p.desc.total_nodes) == (8, 64)
    else:
        assert p.mode == t.MULTI_HIER
        assert (p.desc.side_length, p.desc.total_nodes, p.desc.local_ranks) == (gside, g, L)
        assert p.desc.local_side == local_side
    want = sum(1 << r for r in range(0, 64, L))
    assert p.validated_mask == want
    assert t.multi_plan(["x", "1", "1", "8", "13", "5", "32", "0", "1"], t.BO, gpus=g, check_all=True
                        ).validated_mask == (1 << 64) - 1


def test_plan_mem_and_lo(monkeypatch):
    _env(monkeypatch, 8)
    p = t.multi_plan(["x", "1", "1", "4", "13", "40", "32"], t.MEM, gpus=8)
    assert (p.mode, p.variant, p.desc.variant, p.local_ranks) == (t.MULTI_FLAT, t.MEM, t.MEM, 1)
    p = t.multi_plan(["x", "1", "1", "4", "13", "40", "32"], t.MEM, gpus=1)   # every rank on one GPU
    assert (p.mode, p.local_ranks) == (t.MULTI_LOCAL, 8)
    p = t.multi_plan(["x", "1", "1", "4", "13", "4", "32"], t.LO, gpus=4)       # the legacy LO binary
    assert (p.mode, p.variant, p.desc.variant, p.local_ranks) == (t.MULTI_HIER, t.LO, t.LO, 2)
    p = t.multi_plan(["x", "1", "1", "4", "13", "4", "32", "0", "0"], t.BO, gpus=8)   # bo flag 0 = LO
    assert p.variant == t.LO


def test_plan_refusals_without_gpu(monkeypatch):
    """Impossible splits are refused by the plan, before any HIP call."""
    _env(monkeypatch, 8)
    argv = ["x", "0", "1", "4", "13", "40", "32", "0", "1"]
    for g, err in ((3, t._lib.ERR_ARG), (16, t._lib.ERR_ARG), (0, t._lib.ERR_ARG)):
        with pytest.raises(t.AllredError) as e:
            t.multi_plan(argv, t.BO, gpus=g)
        assert e.value.status == err
    with pytest.raises(t.AllredError) as e:   # mem_2D with several ranks on several GPUs
        t.multi_plan(["x", "1", "1", "4", "13", "40", "32"], t.MEM, gpus=2)
    assert e.value.status == t._lib.ERR_UNSUPPORTED
    with pytest.raises(t.AllredError) as e:   # RCCL cannot put two ranks on one GPU
        t.run_multi(argv, t.BO, gpus=2, transport=t.TRANSPORT_RCCL, share_device=True, outputs=False)
    assert e.value.status == t._lib.ERR_UNSUPPORTED


CASES = [(g, *inv) for g in (2, 4, 8) for inv in invocations(g)]


@pytest.mark.parametrize("g,name,variant,argv,nodes", CASES, ids=[f"g{c[0]}-{c[1]}" for c in CASES])
def test_cli_host_twin_all_values_match(monkeypatch, g, name, variant, argv, nodes):
    """The executable across G 'GPUs' on the host twin: the reference's check at
    ERROR 0 on every rank, under the RNE bfloat16 ctor (its exact expected value)."""
    env = {"ALLRED_TRANSPORT": "host", "ALLRED_GPUS": str(g), "ALLRED_CHECK_ALL": "1", "ALLRED_BF16_ROUND": "rne",
           "ALLRED_STRICT": "1", "ALLRED_REPORT": "1"}
    if nodes is not None:
        env["ALLRED_NODES"] = str(nodes)
    else:
        monkeypatch.delenv("ALLRED_NODES", raising=False)
    r = t.run_cli(BIN[variant], argv_error0(argv, variant), env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "All values match!", r.stdout
    assert '"mismatches": 0' in r.stderr


@pytest.mark.parametrize("g,name,variant,argv,nodes", CASES, ids=[f"g{c[0]}-{c[1]}" for c in CASES])
def test_host_twin_bit_exact_vs_oracle_composition(monkeypatch, g, name, variant, argv, nodes):
    """Arbitrary per-rank data through the same orchestration: every rank's
    result equals the oracle's composition of the plan bit for bit (a wrong
    per-GPU slice, a swapped group or a dropped exchange would show)."""
    _env(monkeypatch, nodes)
    full = ["x", *argv]
    plan = t.multi_plan(full, variant, gpus=g)
    data = random_inputs(plan.total_nodes, int(plan.elems), seed=1000 * g + len(name))
    rep, out = t.run_multi(full, variant, gpus=g, transport=t.TRANSPORT_HOST, inputs=data)
    assert rep.mismatches == -1   # arbitrary data: no closed-form check
    want = expected(plan, data)
    bad = int((out != want).sum())
    assert bad == 0, f"{name} G={g}: {bad} elements differ"


@pytest.mark.parametrize("acc", ["fp32", "bf16"])
def test_host_twin_mem_local_one_gpu(monkeypatch, acc):
    """G = 1 mem_2D: every rank on one GPU, the fused pass (owner first, then
    ranks ascending; fp32 or the reference's bf16 accumulation)."""
    _env(monkeypatch, None)
    if acc == "bf16":
        monkeypatch.setenv("ALLRED_MEM_ACC", "bf16")
    full = ["x", "1", "1", "8", "13", "5", "32"]
    plan = t.multi_plan(full, t.MEM, gpus=1)
    assert plan.mode == t.MULTI_LOCAL
    data = random_inputs(64, int(plan.elems), seed=7)
    rep, out = t.run_multi(full, t.MEM, gpus=1, transport=t.TRANSPORT_HOST, inputs=data)
    assert int((out != expected(plan, data)).sum()) == 0


def test_host_twin_report_and_profile_log(monkeypatch, tmp_path):
    """Report fields and the per-rank ALL_RED_LOOP zones across GPUs."""
    _env(monkeypatch, 8)
    log = tmp_path / "profile_log_device.csv"
    monkeypatch.setenv("ALLRED_PROFILE_LOG", str(log))
    rep, out = t.run_multi(["x", "0", "1", "4", "13", "40", "32", "0", "1"], t.BO, gpus=4,
                           transport=t.TRANSPORT_HOST)
    assert rep.mismatches == 0 and rep.total_nodes == 8 and rep.bytes_per_rank == 655360
    assert rep.device_seconds > 0 and rep.e2e_seconds >= rep.device_seconds
    lines = log.read_text().splitlines()
    assert len(lines) == 2 + 2 * 8 and "ALL_RED_LOOP" in lines[2]
    assert np.array_equal(out[0], out[7])


@pytest.mark.parametrize("g,bad", [(2, 1), (4, 3), (8, 8)])
def test_host_twin_failed_gpu_ends_every_thread(monkeypatch, g, bad):
    """One GPU's thread fails its timed allreduce (tune multi_fault) while the
    others are inside their exchanges: they are cancelled (no waiting for the
    exchange deadline) and the call returns that thread's error — the
    orchestration never hangs on a dead peer."""
    import time
    _env(monkeypatch, None)
    argv = ["x", "1", "1", "8", "13", "5", "32", "0", "1"]
    with t.tuned(multi_fault=bad):
        t0 = time.monotonic()
        with pytest.raises(t.AllredError) as e:
            t.run_multi(argv, t.BO, gpus=g, transport=t.TRANSPORT_HOST, timeout_ms=60000, outputs=False)
        dt = time.monotonic() - t0
    assert e.value.status == t._lib.ERR_TRANSPORT
    assert dt < 20, dt   # cancelled, not the 60 s exchange deadline
    rep, out = t.run_multi(argv, t.BO, gpus=g, transport=t.TRANSPORT_HOST)   # and the next run is fine
    assert rep.mismatches == 0


@pytest.mark.parametrize("g,bad", [(2, 0), (4, 3), (8, 5)])
def test_host_twin_failed_warmup_skips_the_timed_region(monkeypatch, g, bad):
    """One GPU's warm-up fails (tune multi_fault = 33 + GPU): the status
    agreement after the warm-up sends every thread home before the timed
    region (none waits in an exchange with a thread that will not come), and
    the call returns the transport error at once."""
    import time
    _env(monkeypatch, None)
    argv = ["x", "1", "1", "8", "13", "5", "32", "0", "1"]
    with t.tuned(multi_fault=33 + bad):
        t0 = time.monotonic()
        with pytest.raises(t.AllredError) as e:
            t.run_multi(argv, t.BO, gpus=g, transport=t.TRANSPORT_HOST, timeout_ms=60000, outputs=False)
        dt = time.monotonic() - t0
    assert e.value.status == t._lib.ERR_TRANSPORT
    assert dt < 20, dt


@pytest.mark.parametrize("g,bad", [(2, 1), (4, 3)])
def test_host_twin_failed_gpu_skips_its_exchange(monkeypatch, capfd, g, bad):
    """The failed GPU's thread never enters its timed exchange (its reduce is
    skipped, not merely overruled), so every other thread's exchange is ended
    by the cancel, not completed: their timed-launch status is the transport
    error (ALLRED_MULTI_TRACE phases).  Advisor r04: the status guard must skip
    the call itself."""
    _env(monkeypatch, None)
    monkeypatch.setenv("ALLRED_MULTI_TRACE", "1")
    argv = ["x", "1", "1", "8", "13", "5", "32", "0", "1"]
    with t.tuned(multi_fault=bad):
        with pytest.raises(t.AllredError) as e:
            t.run_multi(argv, t.BO, gpus=g, transport=t.TRANSPORT_HOST, timeout_ms=60000, outputs=False)
    assert e.value.status == t._lib.ERR_TRANSPORT
    err = capfd.readouterr().err
    launch = {}
    for line in err.splitlines():
        f = line.split()
        if len(f) >= 6 and f[0] == "multi-trace" and f[2] == "timed-launch":
            launch[int(f[1][1:])] = int(f[-1])
    assert sorted(launch) == list(range(g)), err
    assert all(s == t._lib.ERR_TRANSPORT for s in launch.values()), launch


def test_peer_mem_bf16_refused_before_any_gpu_call(monkeypatch):
    """mem_2D with bf16 accumulation over the peer windows (fp32 only there) is
    refused by allred_run_multi before the backend opens: on this GPU-less
    container the call returns ERR_UNSUPPORTED, not a HIP error."""
    _env(monkeypatch, None)
    monkeypatch.setenv("ALLRED_MEM_ACC", "bf16")
    with pytest.raises(t.AllredError) as e:
        t.run_multi(["x", "1", "1", "4", "13", "40", "32"], t.MEM, gpus=8, transport=t.TRANSPORT_PEER,
                    outputs=False)
    assert e.value.status == t._lib.ERR_UNSUPPORTED
