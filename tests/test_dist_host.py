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
    for variant in ("bo", "lo"):
        for algo in (0, 1):
            out.append((variant, algo, 1))     # flat: one bucket per process
            out.append((variant, algo, 4))     # hierarchical: 4 virtual ranks per process (2x2 local grid)
    return out


def inputs(world, local, n, seed):
    rng = np.random.default_rng(seed)
    return [[rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(local)] for _ in range(world)]


def expected(variant, algo, world, local, data):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    side, total = GRIDS[world]
    if local == 1:
        ranks = [d[0].copy() for d in data]
        oracle.allreduce(variant, algo, side, ranks, total)
        return [[r] for r in ranks]
    partials = []
    for d in data:  # on-GPU tree of local rank 0 (== LO value of local rank 0), Swing 2x2
        loc = [x.copy() for x in d]
        oracle.allreduce("lo", 1, 2, loc, local)
        partials.append(loc[0])
    oracle.allreduce(variant, algo, side, partials, total)
    return [[p.copy() for _ in range(local)] for p in partials]


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    dist.init_process_group("gloo", rank=rank, world_size=world)
    side, total = GRIDS[world]
    n = 8 * total * 16
    fails = []
    for ci, (variant, algo, local) in enumerate(cases(world)):
        data = inputs(world, local, n, seed=100 * world + ci)
        buf = np.concatenate(data[rank]).astype(np.uint16)
        scratch = np.zeros(2 * n, dtype=np.uint16)
        desc = t.dist_desc(algo, t.BO if variant == "bo" else t.LO, side, total, n, local_ranks=local, local_side=2,
                           local_algo=t.SWING)
        t.dist_allreduce_host(desc, rank, buf, scratch, gloo_exchange)
        want = np.concatenate(expected(variant, algo, world, local, data)[rank])
        if not np.array_equal(buf, want):
            fails.append((variant, algo, local, int((buf != want).sum())))
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
