"""The RCCL path on one GPU: a 1-rank communicator (RCCL refuses two ranks on
one device, so N>1 is covered by test_dist_host.py's identical step program
over gloo and by the driver's multi-GPU run).  Checks communicator setup and
the hierarchical stages (on-GPU tree reduce + broadcast) against the host
twin and the oracle, bit for bit."""
import numpy as np
import pytest

import oracle
import tenstorrentallreduce_amd as t

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


# 2,560 elements: one tile per workgroup; 327,680 (config 2, 1,280 tiles) and
# 1,061 tiles (ragged over the 512-workgroup persistent grid): the pipelined form
@pytest.mark.parametrize("n", [64 * 8 * 5, 327680, 1061 * 256])
def test_tree_reduce_and_broadcast_match_oracle(n):
    side, total = 8, 64
    rng = np.random.default_rng(9)
    ranks = [rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(total)]
    buf = torch.from_numpy(np.stack(ranks).view(np.int16)).to(DEV)
    out = torch.empty(n, dtype=torch.int16, device=DEV)
    for algo in (t.SWING, t.RECDUB):
        t.tree_reduce(buf.data_ptr(), n, n, algo, side, total, out.data_ptr())
        torch.cuda.synchronize()
        want = [r.copy() for r in ranks]
        oracle.allreduce("lo", algo, side, want, total)   # LO value of rank 0 = tree of rank 0
        assert np.array_equal(out.cpu().numpy().view(np.uint16), want[0])
    t.broadcast(buf.data_ptr(), n, n, total, out.data_ptr())
    torch.cuda.synchronize()
    got = buf.cpu().numpy().view(np.uint16)
    assert (got == got[0]).all() and np.array_equal(got[0], out.cpu().numpy().view(np.uint16))


@pytest.mark.parametrize("local", [1, 64])
def test_single_rank_rccl_comm(local):
    comm = t.Comm(t.Comm.unique_id(), 1, 0, 0)
    n = 8 * 64 * 4
    rng = np.random.default_rng(local)
    data = [rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(local)]
    buf = torch.from_numpy(np.concatenate(data).view(np.int16)).to(DEV)
    desc = t.dist_desc(t.SWING, t.BO, 1, 1, n, local_ranks=local, local_side=8 if local == 64 else 1,
                       local_algo=t.SWING)
    ws = torch.empty(t.dist_workspace_bytes(desc), dtype=torch.uint8, device=DEV)
    t.dist_allreduce(comm, desc, buf.data_ptr(), ws.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    host = np.concatenate(data).astype(np.uint16)
    scratch = np.zeros(2 * n, dtype=np.uint16)

    def no_exchange(peer, sends, recvs):
        raise AssertionError("a 1-rank grid has no exchange steps")

    t.dist_allreduce_host(desc, 0, host, scratch, no_exchange)
    assert np.array_equal(buf.cpu().numpy().view(np.uint16), host)
    # a bucket or workspace off 16-byte alignment is refused before any exchange
    with pytest.raises(t.AllredError):
        t.dist_allreduce(comm, desc, buf.data_ptr() + 2, ws.data_ptr(), torch.cuda.current_stream())
    with pytest.raises(t.AllredError):
        t.dist_allreduce(comm, desc, buf.data_ptr(), ws.data_ptr() + 8, torch.cuda.current_stream())
    comm.close()


@pytest.mark.parametrize("lag,bal", [(0, 0), (1, 0), (1, 1), (0, 1)])
@pytest.mark.parametrize("n,total,side", [(327680, 64, 8), (64 * 8 * 5, 64, 8), (1061 * 256, 64, 8),
                                          (8 * 8 * 40, 8, 4)])
def test_tree_broadcast_pipelined_matches_the_two_launches(n, total, side, lag, bal):
    """k_tree_bcast_x (bucket i+1's tree and bucket i's broadcast in one pass) is
    bit-identical to tree_reduce(cur) + broadcast(prev); 8 ranks take the two
    launches themselves."""
    rng = np.random.default_rng(n + total)
    cur = torch.from_numpy(rng.integers(0x3F80, 0x42C8, (total, n)).astype(np.uint16).view(np.int16)).to(DEV)
    prev = torch.from_numpy(rng.integers(0x3F80, 0x42C8, (total, n)).astype(np.uint16).view(np.int16)).to(DEV)
    src = torch.from_numpy(rng.integers(0x3F80, 0x42C8, n).astype(np.uint16).view(np.int16)).to(DEV)
    for algo in (t.SWING, t.RECDUB):
        out = torch.empty(n, dtype=torch.int16, device=DEV)
        p2 = prev.clone()
        with t.tuned(tree_bcast_lag=lag, tree_bcast_bal=bal):   # store timing / which waves stage: same bytes
            t.tree_broadcast_pipelined(cur.data_ptr(), p2.data_ptr(), n, n, algo, side, total, out.data_ptr(),
                                       src.data_ptr())
        want = torch.empty_like(out)
        p3 = prev.clone()
        t.tree_reduce(cur.data_ptr(), n, n, algo, side, total, want.data_ptr())
        t.broadcast(p3.data_ptr(), n, n, total, src.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(out, want) and torch.equal(p2, p3)
        assert (p2 == src[None, :]).all()


@pytest.mark.parametrize("buckets", [1, 2, 5])
def test_dist_allreduce_pipelined_one_rank(buckets):
    """allred_dist_allreduce_pipelined over a 1-rank communicator: K buckets in
    K + 1 calls, each bucket bit-identical to allred_dist_allreduce of it; the
    sequence twice (both workspace parities); protocol errors refused."""
    comm = t.Comm(t.Comm.unique_id(), 1, 0, 0)
    n = 327680
    desc = t.dist_desc(t.SWING, t.BO, 1, 1, n, local_ranks=64, local_side=8, local_algo=t.SWING)
    wsb = t.dist_workspace_bytes(desc)
    ws = torch.empty(2 * wsb, dtype=torch.uint8, device=DEV)
    ws1 = torch.empty(wsb, dtype=torch.uint8, device=DEV)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(buckets)
    data = [torch.from_numpy(rng.integers(0x3F80, 0x42C8, (64, n)).astype(np.uint16).view(np.int16)).to(DEV)
            for _ in range(buckets)]
    want = []
    for d in data:
        x = d.clone()
        t.dist_allreduce(comm, desc, x.data_ptr(), ws1.data_ptr(), s)
        want.append(x)
    for _ in range(2):
        got = [d.clone() for d in data]
        for g in got:
            t.dist_allreduce_pipelined(comm, desc, g.data_ptr(), ws.data_ptr(), s)
        t.dist_allreduce_pipelined(comm, desc, None, ws.data_ptr(), s)
        torch.cuda.synchronize()
        for i, (g, w) in enumerate(zip(got, want)):
            assert torch.equal(g, w), i
    with pytest.raises(t.AllredError):   # nothing pending
        t.dist_allreduce_pipelined(comm, desc, None, ws.data_ptr(), s)
    x = data[0].clone()
    t.dist_allreduce_pipelined(comm, desc, x.data_ptr(), ws.data_ptr(), s)
    other = t.dist_desc(t.SWING, t.BO, 1, 1, n // 2, local_ranks=64, local_side=8, local_algo=t.SWING)
    with pytest.raises(t.AllredError):   # another bucket size mid-sequence
        t.dist_allreduce_pipelined(comm, other, x.data_ptr(), ws.data_ptr(), s)
    t.dist_allreduce_pipelined(comm, desc, None, ws.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(x, want[0])
    comm.close()


def test_plain_call_refused_while_a_pipelined_bucket_is_pending():
    """A plain allred_dist_allreduce would overwrite the pending bucket's partial
    in the shared workspace: refused (ALLRED_ERR_ARG) until the flush; so is a
    next bucket overlapping the pending one (k_tree_bcast_x reads cur while it
    writes the pending rows)."""
    comm = t.Comm(t.Comm.unique_id(), 1, 0, 0)
    n = 64 * 8 * 5
    desc = t.dist_desc(t.SWING, t.BO, 1, 1, n, local_ranks=64, local_side=8, local_algo=t.SWING)
    ws = torch.empty(2 * t.dist_workspace_bytes(desc), dtype=torch.uint8, device=DEV)
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(3)
    a = torch.from_numpy(rng.integers(0x3F80, 0x42C8, (64, n)).astype(np.uint16).view(np.int16)).to(DEV)
    b = torch.from_numpy(rng.integers(0x3F80, 0x42C8, (64, n)).astype(np.uint16).view(np.int16)).to(DEV)
    want = a.clone()
    t.dist_allreduce(comm, desc, want.data_ptr(), ws.data_ptr(), s)
    t.dist_allreduce_pipelined(comm, desc, a.data_ptr(), ws.data_ptr(), s)
    for bad in (lambda: t.dist_allreduce(comm, desc, b.data_ptr(), ws.data_ptr(), s),
                lambda: t.dist_allreduce_pipelined(comm, desc, a.data_ptr(), ws.data_ptr(), s),
                lambda: t.dist_allreduce_pipelined(comm, desc, a.data_ptr() + 2 * n, ws.data_ptr(), s)):
        with pytest.raises(t.AllredError) as e:
            bad()
        assert e.value.status == t._lib.ERR_ARG
    t.dist_allreduce_pipelined(comm, desc, None, ws.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(a, want)   # the refused calls touched nothing
    comm.close()


def test_rccl_wait_is_bounded_and_aborts():
    """Bounded RCCL: a wait that never completes — injected with
    tune rccl_fault = 4, as if a partner never arrived — returns
    ALLRED_ERR_TRANSPORT at the deadline, the communicator is aborted
    (ncclCommAbort), and every later call on it refuses (ERR_TRANSPORT)."""
    import time
    comm = t.Comm.init_all([0])[0]
    comm.set_timeout(300)
    n = 8 * 64 * 4
    desc = t.dist_desc(t.SWING, t.BO, 1, 1, n)
    buf = torch.zeros(n, dtype=torch.int16, device=DEV)
    ws = torch.empty(t.dist_workspace_bytes(desc), dtype=torch.uint8, device=DEV)
    s = torch.cuda.current_stream()
    t.dist_allreduce(comm, desc, buf.data_ptr(), ws.data_ptr(), s)
    comm.wait(s)                           # a real drain: fine
    with t.tuned(rccl_fault=4):
        t0 = time.monotonic()
        with pytest.raises(t.AllredError) as e:
            comm.wait(s)
        dt = time.monotonic() - t0
    assert e.value.status == t._lib.ERR_TRANSPORT and 0.25 < dt < 10, dt
    assert comm.aborted
    with pytest.raises(t.AllredError) as e:
        t.dist_allreduce(comm, desc, buf.data_ptr(), ws.data_ptr(), s)
    assert e.value.status == t._lib.ERR_TRANSPORT
    comm.close()


def test_rccl_init_fault_is_bounded():
    """An init that never settles (tune rccl_fault = 1) fails at the operation
    deadline with ALLRED_ERR_TRANSPORT instead of blocking."""
    import time
    with t.tuned(rccl_fault=1):
        t0 = time.monotonic()
        with pytest.raises(t.AllredError) as e:
            t.Comm.init_all([0])
        dt = time.monotonic() - t0
    assert e.value.status == t._lib.ERR_TRANSPORT and dt < 30, dt


def test_rccl_init_with_a_missing_rank_returns_instead_of_hanging():
    """A real missing peer: rank 0 of a 2-rank communicator whose rank 1 never
    joins.  The reference would hang (allred_helper.hpp:84-96); here the
    non-blocking init is aborted at ALLRED_RCCL_INIT_TIMEOUT_MS.  Own process:
    the abort of a half-initialised communicator stays out of the test runner."""
    import os
    import subprocess
    import sys
    import time
    code = ("import tenstorrentallreduce_amd as t\n"
            "try:\n"
            "    t.Comm(t.Comm.unique_id(), 2, 0, 0)\n"
            "    print('joined')\n"
            "except t.AllredError as e:\n"
            "    print('status', e.status)\n")
    env = dict(os.environ, ALLRED_RCCL_INIT_TIMEOUT_MS="3000", ALLRED_RCCL_TIMEOUT_MS="3000",
               PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=90)
    dt = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith(f"status {t._lib.ERR_TRANSPORT}"), (r.stdout, r.stderr[-2000:])
    assert dt < 60, dt


@pytest.mark.parametrize("acc", [t.ACC_FP32, t.ACC_BF16])
def test_mem_2d_over_rccl_across_visible_gpus(acc):
    """mem_2D as an RCCL program across every visible GPU (one thread's worth of
    calls per communicator, ncclCommInitAll-style init): the pairwise rounds,
    the owner-first ordered sum and the gather, bit-exact vs the oracle for fp32
    and the reference's bf16 accumulation.  Needs >= 2 GPUs (skipped on a
    1-GPU box; RCCL refuses two ranks on one device)."""
    import threading
    ng = torch.cuda.device_count()
    if ng < 2:
        pytest.skip("needs >= 2 GPUs")
    ng = 1 << (ng.bit_length() - 1)   # a power of two
    side = {2: 2, 4: 2, 8: 4}[ng]
    n = 8 * ng * 640
    rng = np.random.default_rng(acc + 11)
    data = [rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(ng)]
    comms = t.Comm.init_all(list(range(ng)))
    desc = t.dist_desc(t.SWING, t.MEM, side, ng, n, mem_accum=acc)
    bufs = [torch.from_numpy(d.view(np.int16)).to(f"cuda:{g}") for g, d in enumerate(data)]
    wss = [torch.empty(t.dist_workspace_bytes(desc), dtype=torch.uint8, device=f"cuda:{g}") for g in range(ng)]
    errs = []

    def one(g):
        try:
            torch.cuda.set_device(g)
            s = torch.cuda.current_stream(g)
            t.dist_allreduce(comms[g], desc, bufs[g].data_ptr(), wss[g].data_ptr(), s)
            comms[g].wait(s)
        except Exception as e:  # reported below
            errs.append(repr(e))

    th = [threading.Thread(target=one, args=(g,)) for g in range(ng)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=60)
    assert not errs, errs
    want = [d.copy() for d in data]
    oracle.allreduce("mem", t.SWING, side, want, ng, acc == t.ACC_BF16)
    for g in range(ng):
        assert np.array_equal(bufs[g].cpu().numpy().view(np.uint16), want[g]), g
    for c in comms:
        c.close()
