"""The multi-GPU step program (dist.cpp) on CPU: world_size 2/4/8 processes over
gloo, the library's allred_dist_allreduce_host twin with a gloo exchange.
It runs the identical per-rank program the RCCL path runs (same partners,
same block runs in the same order, same adds), so this covers every step of
the N>1 path; results must equal the oracle's bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GRIDS = {2: (2, 2), 4: (2, 4), 8: (4, 8)}


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


def cases(world):
    out = []
    cmax = world - 1  # 2^S - 1 link-spreading channels on the XOR grids
    for variant in ("bo", "lo"):
        out.append((variant, 3, 1, 1))             # 1D Swing prototype schedule (no channels: not XOR)
        out.append((variant, 2, 1, cmax))          # 1D RecDub (an XOR schedule)
        for algo in (0, 1):
            out.append((variant, algo, 1, 1))      # flat: one bucket per process
            out.append((variant, algo, 4, 1))      # hierarchical: 4 virtual ranks per process (2x2 local grid)
            if cmax > 1:
                out.append((variant, algo, 1, cmax))   # every link at every step
                out.append((variant, algo, 4, 2))      # fewer channels than links
    return out


def gf_mul(a, b, S):
    poly = {1: 0x3, 2: 0x7, 3: 0xB}[S]
    r = 0
    for i in range(S):
        if (b >> i) & 1:
            r ^= a << i
    for i in range(2 * S - 2, S - 1, -1):
        if (r >> i) & 1:
            r ^= poly << (i - S)
    return r


def slices(n, N, C):
    unit = 8 * N
    units = n // unit
    q, rem = divmod(units, C)
    out, start = [], 0
    for c in range(C):
        ln = (q + (1 if c < rem else 0)) * unit
        out.append((start, ln))
        start += ln
    return out


def inputs(world, local, n, seed):
    rng = np.random.default_rng(seed)
    return [[rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(local)] for _ in range(world)]


def channel_allreduce(oracle, variant, algo, side, total, vecs, C):
    """C link-spreading channels: channel c allreduces its slice with rank r
    relabelled as a^c * r in GF(2^S) (a = x), i.e. the plain schedule run on
    the permuted ranks."""
    if algo >= 2:
        side = 1
    if C == 1:
        oracle.allreduce(variant, algo, side, vecs, total)
        return
    S = total.bit_length() - 1
    for c, (b0, ln) in enumerate(slices(vecs[0].size, total, C)):
        a = 1
        for _ in range(c):
            a = gf_mul(a, 2, S)
        lab = [gf_mul(a, r, S) for r in range(total)]
        base = [None] * total
        for r in range(total):
            base[lab[r]] = vecs[r][b0:b0 + ln].copy()
        oracle.allreduce(variant, algo, side, base, total)
        for r in range(total):
            vecs[r][b0:b0 + ln] = base[lab[r]]


def expected(variant, algo, world, local, data, C):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    side, total = GRIDS[world]
    if local == 1:
        ranks = [d[0].copy() for d in data]
        channel_allreduce(oracle, variant, algo, side, total, ranks, C)
        return [[r] for r in ranks]
    partials = []
    for d in data:  # on-GPU tree of local rank 0 (== LO value of local rank 0), Swing 2x2
        loc = [x.copy() for x in d]
        oracle.allreduce("lo", 1, 2, loc, local)
        partials.append(loc[0])
    channel_allreduce(oracle, variant, algo, side, total, partials, C)
    return [[p.copy() for _ in range(local)] for p in partials]


def mem_worker(rank, world, port, q):
    """mem_2D over the RCCL program (local_ranks == 1): the pairwise all-to-all
    rounds, the owner's ordered sum (own copy first, then ranks in order; fp32
    rounded once, or the reference's bf16 accumulation), the all-gather — the
    host twin over gloo bit-exact against the oracle's allred_mem_2D restatement."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import tenstorrentallreduce_amd as t
    dist.init_process_group("gloo", rank=rank, world_size=world)
    side, total = GRIDS[world]
    n = 8 * total * 24
    fails = []
    for acc in (t.ACC_FP32, t.ACC_BF16):
        data = inputs(world, 1, n, seed=900 + 10 * world + acc)
        buf = data[rank][0].copy()
        scratch = np.zeros(2 * n, dtype=np.uint16)
        desc = t.dist_desc(t.SWING, t.MEM, side, total, n, mem_accum=acc)
        t.dist_allreduce_host(desc, rank, buf, scratch, gloo_exchange)
        want = [d[0].copy() for d in data]
        oracle.allreduce("mem", 1, side, want, total, acc16=acc == t.ACC_BF16)
        if not np.array_equal(buf, want[rank]):
            fails.append((acc, int((buf != want[rank]).sum())))
    st = t.dist_program_stats(t.dist_desc(t.SWING, t.MEM, side, total, n), rank)
    if st != {"steps": 2, "add_launches": 1, "segments": 4 * (world - 1)}:
        fails.append(("stats", st))
    try:   # hierarchical mem_2D is not an RCCL program
        t.dist_allreduce_host(t.dist_desc(t.SWING, t.MEM, side, total, n, local_ranks=4, local_side=2), rank,
                              np.zeros(4 * n, np.uint16), np.zeros(2 * n, np.uint16), gloo_exchange)
        fails.append("hierarchical mem accepted")
    except t.AllredError:
        pass
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, fails))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_mem_program_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=mem_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, fails in results:
        assert fails == [], (rank, fails)


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    dist.init_process_group("gloo", rank=rank, world_size=world)
    side, total = GRIDS[world]
    n = 8 * total * 16
    fails = []
    for ci, (variant, algo, local, chans) in enumerate(cases(world)):
        data = inputs(world, local, n, seed=100 * world + ci)
        buf = np.concatenate(data[rank]).astype(np.uint16)
        scratch = np.zeros(2 * n, dtype=np.uint16)
        desc = t.dist_desc(algo, t.BO if variant == "bo" else t.LO, 1 if algo >= 2 else side, total, n,
                           local_ranks=local, local_side=2,
                           local_algo=t.SWING, channels=chans)
        t.dist_allreduce_host(desc, rank, buf, scratch, gloo_exchange)
        want = np.concatenate(expected(variant, algo, world, local, data, chans)[rank])
        if not np.array_equal(buf, want):
            fails.append((variant, algo, local, chans, int((buf != want).sum())))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, fails))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dist_program_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, fails in results:
        assert fails == [], (rank, fails)


def test_dist_desc_validation():
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    buf = np.zeros(8 * 8 * 4, dtype=np.uint16)
    scratch = np.zeros_like(buf)
    bad = t.dist_desc(t.SWING, t.BO, 8, 16, buf.size)        # invalid rectangle
    with pytest.raises(t.AllredError):
        t.dist_allreduce_host(bad, 0, buf, scratch, gloo_exchange)
    bad = t.dist_desc(t.SWING, t.BO, 4, 8, 100)              # not a multiple of 8 * total
    with pytest.raises(t.AllredError):
        t.dist_allreduce_host(bad, 0, buf, scratch, gloo_exchange)


# ------------------------------------------------------------------ check mode
def check_worker(rank, world, port, q):
    """tune check=1: the same programs verified against the partners' and run
    with every receive region poisoned (0xFFFF) first — results stay bit-exact;
    then fault injection: the exchange silently drops one received run at one
    rank.  Without the check mode the result is stale data that passes as
    numbers; with it the dropped elements come out as NaN (detected)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    dist.init_process_group("gloo", rank=rank, world_size=world)
    side, total = GRIDS[world]
    n = 8 * total * 16
    out = {}
    with t.tuned(check=1):
        for ci, (variant, algo, local, chans) in enumerate(cases(world)):
            data = inputs(world, local, n, seed=300 * world + ci)
            buf = np.concatenate(data[rank]).astype(np.uint16)
            scratch = np.zeros(2 * n, dtype=np.uint16)
            desc = t.dist_desc(algo, t.BO if variant == "bo" else t.LO, 1 if algo >= 2 else side, total, n,
                               local_ranks=local, local_side=2, local_algo=t.SWING, channels=chans)
            t.dist_allreduce_host(desc, rank, buf, scratch, gloo_exchange)
            want = np.concatenate(expected(variant, algo, world, local, data, chans)[rank])
            out.setdefault("exact", []).append(bool(np.array_equal(buf, want)))

    calls = [0]

    def dropping_exchange(peer, sends, recvs):   # rank 0 loses its first received run of the first step
        tmps = [torch.from_numpy(v.copy()) for v in recvs]
        reqs = [dist.isend(torch.from_numpy(v), peer, tag=i) for i, v in enumerate(sends)]
        reqs += [dist.irecv(x, peer, tag=i) for i, x in enumerate(tmps)]
        for r in reqs:
            r.wait()
        for i, (v, x) in enumerate(zip(recvs, tmps)):
            if not (rank == 0 and calls[0] == 0 and i == 0):
                v[:] = x.numpy()
        calls[0] += 1

    for check in (0, 1):
        calls[0] = 0
        data = inputs(world, 1, n, seed=77)
        buf = data[rank][0].copy()
        scratch = np.zeros(2 * n, dtype=np.uint16)
        desc = t.dist_desc(t.SWING, t.BO, side, total, n)
        with t.tuned(check=check):
            t.dist_allreduce_host(desc, rank, buf, scratch, dropping_exchange)
        f = (buf.astype(np.uint32) << 16).view(np.float32)
        want = expected("bo", t.SWING, world, 1, data, 1)[rank][0]
        out[f"check{check}"] = (int(np.isnan(f).sum()), int((buf != want).sum()))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 4])
def test_check_mode_poison_and_fault_injection(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=check_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in results.items():
        assert all(out["exact"]), (rank, out["exact"])
    # the dropped run corrupts results (somewhere) either way; only the check mode makes it NaN
    assert sum(out["check0"][1] for out in results.values()) > 0
    assert all(out["check0"][0] == 0 for out in results.values())
    assert sum(out["check1"][0] for out in results.values()) > 0
    assert all(out["check1"][0] == out["check1"][1] for out in results.values())
