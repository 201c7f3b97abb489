"""bench.py's N > 1 verification without a GPU: verify_transport runs the
library's host twin of the RCCL program (allred_dist_allreduce_host, the same
per-rank step program) over gloo with world 2 and 4, passes both independent
checks (exact sums of 0/1 inputs, the reference's closed form RNE(a+b)*R/2), and
refuses deliberately corrupted programs; an unverified transport or arm never
becomes the headline or the xGMI roofline."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

GRIDS = {2: (2, 2), 4: (2, 4)}


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def gloo_exchange(peer, sends, recvs):
    reqs = [dist.isend(torch.from_numpy(v), peer, tag=i) for i, v in enumerate(sends)]
    reqs += [dist.irecv(torch.from_numpy(v), peer, tag=i) for i, v in enumerate(recvs)]
    for r in reqs:
        r.wait()


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    dist.init_process_group("gloo", rank=rank, world_size=world)
    side, total = GRIDS[world]
    out = {}
    cases = [("bo_hier", t.SWING, t.BO, 4, 2), ("lo_flat", t.SWING, t.LO, 1, 1), ("recdub_flat", t.RECDUB, t.BO, 1, 1),
             ("mem_flat", t.SWING, t.MEM, 1, 1), ("bo_hier_64", t.SWING, t.BO, 64, 8)]
    for name, algo, variant, local, lside in cases:
        n = 8 * total * 32
        desc = t.dist_desc(algo, variant, side, total, n, local_ranks=local, local_side=lside, local_algo=t.SWING)

        def run(b, exchange=gloo_exchange, corrupt=False):
            flat = b.numpy().reshape(-1).view(np.uint16)
            scratch = np.zeros(2 * n, dtype=np.uint16)
            t.dist_allreduce_host(desc, rank, flat, scratch, exchange)
            if corrupt and rank == world - 1:   # one element off by one bf16 ulp on one rank
                flat[n // 2 + 3] ^= 1

        buf = torch.empty((local, n), dtype=torch.int16)
        out[name] = bench.verify_transport(run, buf, world, rank, local, lside, side, seed=100 + len(out))
        out[name + "_corrupt"] = bench.verify_transport(lambda b: run(b, corrupt=True), buf, world, rank, local,
                                                        lside, side, seed=200 + len(out))

    calls = [0]

    def dropping_exchange(peer, sends, recvs):   # rank 0 silently loses its first received run
        tmps = [torch.from_numpy(v.copy()) for v in recvs]
        reqs = [dist.isend(torch.from_numpy(v), peer, tag=i) for i, v in enumerate(sends)]
        reqs += [dist.irecv(x, peer, tag=i) for i, x in enumerate(tmps)]
        for r in reqs:
            r.wait()
        for i, (v, x) in enumerate(zip(recvs, tmps)):
            if not (rank == 0 and calls[0] == 0 and i == 0):
                v[:] = x.numpy()
        calls[0] += 1

    n = 8 * total * 32
    desc = t.dist_desc(t.SWING, t.BO, side, total, n)

    def run_drop(b):
        calls[0] = 0
        flat = b.numpy().reshape(-1).view(np.uint16)
        t.dist_allreduce_host(desc, rank, flat, np.zeros(2 * n, np.uint16), dropping_exchange)

    out["dropped_run"] = bench.verify_transport(run_drop, torch.empty((1, n), dtype=torch.int16), world, rank, 1, 1,
                                                side, seed=300)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 4])
def test_verify_transport_accepts_correct_and_refuses_corrupted(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in results.items():
        for name, v in out.items():
            if name.endswith("_corrupt") or name == "dropped_run":
                assert v["verified"] is False, (rank, name, v)   # every rank refuses it (agreed)
            else:
                assert v == {"exact_sum": True, "closed_form": True, "verified": True}, (rank, name, v)
        assert "error" not in out["bo_hier_corrupt"]   # a wrong result, not a refused call
        assert out["bo_hier_corrupt"]["exact_sum"] is False and out["bo_hier_corrupt"]["closed_form"] is False


def test_exact_inputs_are_exact_and_rank_independent():
    """Every rank evaluates every row's 0/1 inputs; their sum fits bf16 exactly."""
    n, rows = 4096, 512
    want = bench.exact_expected(rows, n, 7, "cpu").view(torch.bfloat16).float()
    acc = torch.zeros(n)
    tmp = torch.empty(n, dtype=torch.int16)
    for r in range(rows):
        bench.exact_bits_(tmp, r, 7)
        acc += tmp.view(torch.bfloat16).float()
    assert torch.equal(acc, want) and 64 < acc.mean() < 192
    bench.exact_bits_(tmp, 3, 7)
    again = torch.empty_like(tmp)
    bench.exact_bits_(again, 3, 7)
    other = torch.empty_like(tmp)
    bench.exact_bits_(other, 4, 7)
    assert torch.equal(tmp, again) and not torch.equal(tmp, other)


def test_closed_form_is_the_references_expected_value():
    """RNE(a+b)*R/2 == validate_result_vector's expected bf16((a+b)*(R/2)) under the RNE ctor."""
    a, b = bench.ref_pair(1 << 14, 5, "cpu")
    cf = bench.closed_form(a, b, 64).view(torch.bfloat16).float()
    ref = ((a.float() + b.float()) * 32).to(torch.bfloat16).float()
    assert torch.equal(cf, ref)


def test_dropped_candidates_are_listed_with_a_reason():
    """xgmi.dropped: a form that failed verification or whose quick timing had a
    peer wait give up is listed (and never chosen); verified forms are not."""
    verify = {"rccl": {"verified": True, "exact_sum": True, "closed_form": True},
              "peer_hier_x": {"verified": False, "quick_timing_timeout": True},
              "peer_hier_ws": {"verified": False, "exact_sum": True, "closed_form": True,
                               "matches_peer_launches": False},
              "peer_swing": {"verified": False, "exact_sum": False, "closed_form": True},
              "peer_hier_ws_fenced": {"verified": True, "exact_sum": True, "closed_form": True,
                                     "matches_peer_launches": True}}
    quick = {"rccl": 1.0, "peer_hier_ws_fenced": 0.6}
    assert bench.choose_transport(quick, verify) == "peer_hier_ws_fenced"
    got = {d["transport"]: d["reason"] for d in bench.dropped_candidates(verify)}
    assert set(got) == {"peer_hier_x", "peer_hier_ws", "peer_swing"}
    assert got["peer_hier_x"].startswith("quick_timing_timeout")
    assert got["peer_hier_ws"] == "differs from peer_launches"
    assert got["peer_swing"] == "exact_sum check failed"
    assert bench.dropped_candidates({"rccl": {"verified": True}}) == []


def test_unverified_never_headline_nor_roofline():
    quick = {"rccl": 1.0, "peer_hier_ws": 0.5, "peer_swing": 0.8}
    verify = {"rccl": {"verified": True}, "peer_hier_ws": {"verified": False}, "peer_swing": {"verified": True}}
    assert bench.choose_transport(quick, verify) == "peer_swing"
    assert bench.choose_transport(quick, {}) is None
    arm = "config4_swing_bo_1GiB_all_links"
    extras = {arm: {"busbw_GBps": 300.0, "verified": True}, "peer_" + arm: {"busbw_GBps": 900.0, "verified": False},
              "link_probe": {"GBps_per_direction": 64.0}}
    r = bench.roofline_xgmi(extras, 8)
    assert r["arm"] == arm and r["achieved"] == 300.0 and r["frac"] == round(300 / (7 * 64.0), 4)
    extras[arm]["busbw_GBps"] = 500.0            # above the measured peak: no fraction is claimed
    r = bench.roofline_xgmi(extras, 8)
    assert r["frac"] is None and r["frac_unbounded"] > 1
    del extras["link_probe"]                      # no measured link: frac null, spec figure beside it
    r = bench.roofline_xgmi(extras, 8)
    assert r["frac"] is None and r["peak"] is None and r["frac_spec"] > 0
    extras[arm]["verified"] = False
    assert bench.roofline_xgmi(extras, 8)["achieved"] is None


def comparator_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out = bench.rccl_allreduce_comparator(rank, world, "cpu", backend="gloo",
                                             sizes=(("small", 8 * 1024 * 2, 3), ("odd", 3000 * 2, 2)))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, {"exception": repr(e), "tb": traceback.format_exc()}))


@pytest.mark.parametrize("world", [2, 4])
def test_rccl_allreduce_comparator_verifies_and_reports_busbw(world):
    """The N > 1 line's RCCL ncclAllReduce comparator (an external comparator,
    never the product path) run over gloo on CPU: each size is verified exact on small integers
    before it is timed, and reports busbw like the arms."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=comparator_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, out in results.items():
        assert "exception" not in out, out
        for name in ("small", "odd"):
            v = out[name]
            assert v["verified_exact"] is True and v["ms"] > 0 and v["busbw_GBps"] > 0, v
