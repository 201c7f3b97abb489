"""Peer-mapped one-shot allreduce (allred_peer_*, the mem_2D variant over
IPC-mapped windows) with 2 and 4 processes sharing ONE MI355X: the same code
path as across GPUs (IPC handles, uncached flag words, system-scope atomics,
parity-double-buffered windows), with real cross-process concurrency.
Results must equal the oracle's mem_2D semantics bit for bit, over several
consecutive calls (epochs and window parities)."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def placement(rank, world, devs, tunes):
    """A worker's device (devs[rank]; None: every rank on device 0, the one-GPU
    rehearsal) and the tune keys every rank sets before its first call
    (bit-identical forms, e.g. peer_fence).  Returns (devs, "cuda:i", shared)."""
    import tenstorrentallreduce_amd as t
    devs = list(devs) if devs else [0] * world
    torch.cuda.set_device(devs[rank])
    for k, v in (tunes or {}).items():
        t.tune(k, v)
    return devs, f"cuda:{devs[rank]}", len(set(devs)) < world


def run_world(target, world, timeout, devs=None, tunes=None):
    """world spawned processes running target(rank, world, port, q, devs, tunes);
    every rank must report no failure and a clean peer status word."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q, devs, tunes)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in procs:
            results.append(q.get(timeout=timeout))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, fails, status in results:
        assert fails == [], (rank, fails)
        assert status == 0, (rank, status)


def worker(rank, world, port, q, devs=None, tunes=None):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import tenstorrentallreduce_amd as t
        import oracle
        devs, dev, shared = placement(rank, world, devs, tunes)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        unit = 8 * world
        sizes = [unit, unit * 64 * 5, unit * 3, unit * 8200, unit * 64 * 5]   # 8200 vectors: > 128 groups x 64
        n = unit * 64 * 5
        peer = t.Peer(world, rank, devs[rank], max(sizes))
        handles = [None] * world
        dist.all_gather_object(handles, peer.handle())
        peer.connect(handles)
        # the one-kernel forms wait across processes: every process's grid must be
        # resident at once on the shared GPU (one GPU per process needs no cap)
        peer.set_max_groups(256 // world if shared else 0)
        fails = []
        call = 0
        for mode, limit, ll_max in (("oneshot", 1 << 40, 0), ("steps", 0, 0), ("auto", 1 << 20, 256 << 10),
                                    ("ll", 0, 1 << 40)):
            peer.set_oneshot_max(limit)
            peer.set_mem_ll_max(ll_max)   # k_peer_mem_ll where the LL area holds the bucket
            for m in sizes:
                rng = [np.random.default_rng(1000 * call + r) for r in range(world)]
                data = [g.integers(0x3F80, 0x42C8, m).astype(np.uint16) for g in rng]
                buf = torch.from_numpy(data[rank].view(np.int16)).to(dev)
                peer.allreduce(buf.data_ptr(), m, torch.cuda.current_stream())
                torch.cuda.synchronize()
                want = [d.copy() for d in data]
                oracle.allreduce("mem", 0, 1, want, world)
                got = buf.cpu().numpy().view(np.uint16)
                if not np.array_equal(got, want[rank]):
                    fails.append((mode, m, call, int((got != want[rank]).sum()), peer.status()))
                call += 1
                dist.barrier()
        # back-to-back calls with no host sync in between (window parities, epochs)
        bufs = []
        for k in range(6):
            d = np.random.default_rng(50 + k * world + rank).integers(0x3F80, 0x42C8, n).astype(np.uint16)
            bufs.append(torch.from_numpy(d.view(np.int16)).to(dev))
        torch.cuda.synchronize()
        dist.barrier()
        for k, b in enumerate(bufs):   # launches / one kernel / LL pushes, interleaved
            peer.set_oneshot_max(1 << 40 if k % 2 else 0)
            peer.set_mem_ll_max(1 << 40 if k % 3 == 2 else 0)
            peer.allreduce(b.data_ptr(), n, torch.cuda.current_stream())
        torch.cuda.synchronize()
        for k, b in enumerate(bufs):
            want = [np.random.default_rng(50 + k * world + r).integers(0x3F80, 0x42C8, n).astype(np.uint16)
                    for r in range(world)]
            oracle.allreduce("mem", 0, 1, want, world)
            if not np.array_equal(b.cpu().numpy().view(np.uint16), want[rank]):
                fails.append(("pipelined", k))
        dist.barrier()
        peer.set_mem_ll_max(0)   # the forms below as before (LL mem_2D is covered above)
        # hierarchical: 8 virtual ranks per process (4x2 Swing local grid)
        local = 8
        data = [np.random.default_rng(77 + r).integers(0x3F80, 0x42C8, (local, n)).astype(np.uint16)
                for r in range(world)]
        buf = torch.from_numpy(data[rank].view(np.int16)).to(dev)
        ws = torch.empty(n, dtype=torch.int16, device=dev)
        peer.allreduce(buf.data_ptr(), n, torch.cuda.current_stream(), local, 4, t.SWING, ws.data_ptr())
        torch.cuda.synchronize()
        partials = []
        for d in data:
            loc = [x.copy() for x in d]
            oracle.allreduce("lo", 1, 4, loc, local)   # tree of local rank 0
            partials.append(loc[0])
        oracle.allreduce("mem", 0, 1, partials, world)
        got = buf.cpu().numpy().view(np.uint16)
        if not all(np.array_equal(got[i], partials[rank]) for i in range(local)):
            fails.append(("hier", 0, 1))
        # 64 local ranks (8x8 Swing tree per GPU): the one-kernel hierarchical form with LL push
        # hand-offs (k_hier_ws), the launch form (the mem_2D exchange as one kernel or as launches)
        # and the two-deep bucket pipeline (k_hier_x2), two or three calls back to back each (then
        # k_hier_ws once more after the launch form: its boxes must not accept the older calls' words)
        local, m = 64, 256 * world * 3
        # in full and capped grids (a capped grid gives every workgroup many tiles)
        for mi, (mode, limit, ll, cap, *more) in enumerate((("hier_oneshot_exchange", 1 << 40, 0, 0),
                                                     ("hier_launches", 0, 0, 0), ("hier_oneshot_exchange_capped", 1 << 40, 0, 1),
                                                     # k_hier_ws; one workgroup with 20 tiles per owner: owned
                                                     # partials past its 16 LDS slots go through the own inbox
                                                     ("hier_ws", 0, 1, 0), ("hier_ws_capped", 0, 1, 2),
                                                     ("hier_launches_then_ws", 0, 0, 0), ("hier_ws_again", 0, 1, 0),
                                                     ("hier_ws_ring", 0, 1, 1, 20), ("hier_ws_c8", 0, 1, 0),
                                                     ("hier_ws_c8_ring", 0, 1, 1, 20), ("hier_ws_c32", 0, 1, 0),
                                                     ("hier_ws_c32_ring", 0, 1, 1, 20),
                                                     ("hier_x2", 0, 0, 0), ("hier_x2_capped", 0, 0, -1),
                                                     # one workgroup: 3 * world tiles, results staged 8 at a time
                                                     # (two chunks resident, the third reusing the first's slot)
                                                     ("hier_x2_one_group", 0, 0, 1),
                                                     ("hier_ws_after_x2", 0, 1, 0))):
            m = 256 * world * (more[0] if more else 3)
            if cap < 0:   # exactly 8 tiles per workgroup: one chunk of k_hier_x2
                cap = (m // 256 + 7) // 8
            peer.set_oneshot_max(limit)
            peer.set_hier_ll(ll)
            peer.set_max_groups(cap)
            runs = []
            for rep in range(3 if mode.startswith("hier_x2") else 2):   # x2: one launch with cur, mid and old
                data = [np.random.default_rng(700 + 100 * mi + 10 * rep + r).integers(0x3F80, 0x42C8, (local, m)).astype(np.uint16)
                        for r in range(world)]
                buf = torch.from_numpy(data[rank].view(np.int16)).to(dev)
                ws = torch.empty(m, dtype=torch.int16, device=dev)
                if mode.startswith("hier_x2"):   # two deep: b0, b1, b2, then the flush below
                    peer.allreduce_pipelined2(buf.data_ptr(), m, torch.cuda.current_stream())
                else:
                    with t.tuned(hier_ws_cols=8 if "_c8" in mode else 32 if "_c32" in mode else 16):
                        peer.allreduce(buf.data_ptr(), m, torch.cuda.current_stream(), local, 8, t.SWING, ws.data_ptr())
                runs.append((data, buf, ws))
            if mode.startswith("hier_x2"):
                peer.allreduce_pipelined2(None, m, torch.cuda.current_stream())
            torch.cuda.synchronize()
            for rep, (data, buf, _) in enumerate(runs):
                partials = []
                for d in data:
                    loc = [x.copy() for x in d]
                    oracle.allreduce("lo", 1, 8, loc, local)   # tree of local rank 0
                    partials.append(loc[0])
                oracle.allreduce("mem", 0, 1, partials, world)
                got = buf.cpu().numpy().view(np.uint16)
                bad = sum(int((got[i] != partials[rank]).sum()) for i in range(local))
                if bad:
                    fails.append((mode, rep, bad))
            if peer.status() & t.PEER_TIMEOUT and not any(f[0] == "timeout" for f in fails):
                fails.append(("timeout", mode, 0))   # the first mode whose peer waits gave up
            dist.barrier()
        peer.set_hier_ll(0)
        peer.set_max_groups(0)
        status = peer.status()
        dist.barrier()
        peer.close()
        dist.destroy_process_group()
        q.put((rank, fails, status))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())], -1))


# tune peer_fence = 1: a system-scope release fence before every cross-GPU hand-off store and an
# acquire fence after every wait (the same bits)
FENCES = pytest.mark.parametrize("tunes", [{}, {"peer_fence": 1}], ids=["relaxed", "fenced"])


@FENCES
@pytest.mark.parametrize("world", [2, 4, 8])
def test_peer_one_shot_multi_process_one_gpu(world, tunes):
    run_world(worker, world, 240, tunes=tunes)


def dist_worker(rank, world, port, q, devs=None, tunes=None):
    """allred_peer_dist_allreduce: every case of the gloo-tested RCCL program
    (tests/test_dist_host.py: Swing / RecDub / 1D schedules, BO and LO, flat and
    hierarchical, link-spreading channels) over the peer windows — read by the
    receiver (k_peer_sched), pushed by the sender (k_peer_sched_push, BO), LL
    (k_peer_lo_ll, small LO) — bit-exact with the oracle; each case twice back
    to back, a mem_2D call in between."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import tenstorrentallreduce_amd as t
        import test_dist_host as tdh
        devs, dev, shared = placement(rank, world, devs, tunes)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        side, total = tdh.GRIDS[world]
        n = 8 * total * 16 * 3
        peer = t.Peer(world, rank, devs[rank], 4 * n * 2)
        handles = [None] * world
        dist.all_gather_object(handles, peer.handle())
        peer.connect(handles)
        fails = []
        # LO buckets this small take the LL-push program by default (k_peer_lo_ll);
        # the second pass forces the scheduled form (k_peer_sched) for every case, the
        # third its push form (k_peer_sched_push) for every BO case
        for ci, (variant, algo, local, chans, ll_max, push) in enumerate(
                [c + (256 << 10, 0) for c in tdh.cases(world)] + [c + (0, 0) for c in tdh.cases(world)] +
                [c + (0, 1) for c in tdh.cases(world) if c[0] == "bo"]):
            peer.set_lo_ll_max(ll_max)
            peer.set_sched_push(push)
            desc = t.dist_desc(algo, t.BO if variant == "bo" else t.LO, 1 if algo >= 2 else side, total, n,
                               local_ranks=local, local_side=2, local_algo=t.SWING, channels=chans)
            ws = torch.empty(max(t.dist_workspace_bytes(desc), 16), dtype=torch.uint8, device=dev)
            runs = []
            for rep in range(2):
                data = tdh.inputs(world, local, n, seed=1000 * world + 10 * ci + rep)
                buf = torch.from_numpy(np.concatenate(data[rank]).view(np.int16)).to(dev)
                peer.dist_allreduce(desc, buf.data_ptr(), ws.data_ptr(), torch.cuda.current_stream())
                runs.append((data, buf))
            torch.cuda.synchronize()
            for rep, (data, buf) in enumerate(runs):
                want = np.concatenate(tdh.expected(variant, algo, world, local, data, chans)[rank])
                got = buf.cpu().numpy().view(np.uint16)
                if not np.array_equal(got, want):
                    fails.append((variant, algo, local, chans, ll_max, push, rep, int((got != want).sum())))
            # a mem_2D call (reads every window) between scheduled calls
            m = torch.zeros(n, dtype=torch.int16, device=dev)
            peer.allreduce(m.data_ptr(), n, torch.cuda.current_stream())
        torch.cuda.synchronize()
        status = peer.status()
        dist.barrier()
        peer.close()
        dist.destroy_process_group()
        q.put((rank, fails, status))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())], -1))


@FENCES
@pytest.mark.parametrize("world", [2, 4, 8])
def test_peer_scheduled_program_multi_process_one_gpu(world, tunes):
    run_world(dist_worker, world, 300, tunes=tunes)


def skew_worker(rank, world, port, q, devs=None, tunes=None):
    """The hierarchical hand-offs under launch skew: before each call every process queues a
    spin of a random length (per rank and call, 0-300 us: up to twenty kernels' time) on its
    stream, so the processes' launches run out of step — 12 back-to-back k_hier_ws calls, then
    a k_hier_x2 sequence of 8 buckets with the same skew between its calls.  Every bucket must
    equal the oracle's composition bit for bit: a launch may overwrite a parity's hand-off
    slots only once every consumer of that parity's previous call is done, and
    skew is what would break a protocol that leans on the processes running in step."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import tenstorrentallreduce_amd as t
        import oracle
        import bench
        devs, dev, shared = placement(rank, world, devs, tunes)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        local, m = 64, 256 * world * 4
        peer = t.Peer(world, rank, devs[rank], m)
        handles = [None] * world
        dist.all_gather_object(handles, peer.handle())
        peer.connect(handles)
        peer.set_max_groups(256 // world if shared else 0)
        peer.set_hier_ll(1)
        s = torch.cuda.current_stream()
        cyc = bench.spin_cycles_per_us(s)
        rng = np.random.default_rng(4242 + rank)

        def data(c, r):
            return np.random.default_rng(6000 + 100 * c + r).integers(0x3F80, 0x42C8, (local, m)).astype(np.uint16)

        def expected(c):
            partials = []
            for r in range(world):
                loc = [x.copy() for x in data(c, r)]
                oracle.allreduce("lo", 1, 8, loc, local)   # tree of local rank 0
                partials.append(loc[0])
            oracle.allreduce("mem", 0, 1, partials, world)
            return partials[rank]

        def skew():
            torch.cuda._sleep(int(rng.integers(0, 300) * cyc))

        fails = []
        ws = torch.empty(m, dtype=torch.int16, device=dev)
        bufs = [torch.from_numpy(data(c, rank).view(np.int16)).to(dev) for c in range(20)]
        torch.cuda.synchronize()
        dist.barrier()
        for c in range(12):   # k_hier_ws, one launch per bucket
            skew()
            peer.allreduce(bufs[c].data_ptr(), m, s, local, 8, t.SWING, ws.data_ptr())
        for c in range(12, 20):   # k_hier_x2, two buckets deep
            skew()
            peer.allreduce_pipelined2(bufs[c].data_ptr(), m, s)
        skew()
        peer.allreduce_pipelined2(None, m, s)
        torch.cuda.synchronize()
        for c, b in enumerate(bufs):
            bad = int((b.cpu().numpy().view(np.uint16) != expected(c)[None, :]).sum())
            if bad:
                fails.append(("skew", c, bad))
        status = peer.status()
        dist.barrier()
        peer.set_hier_ll(0)
        peer.close()
        dist.destroy_process_group()
        q.put((rank, fails, status))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())], -1))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_hier_handoffs_under_launch_skew_one_gpu(world):
    run_world(skew_worker, world, 300)


def skew_flat_worker(rank, world, port, q, devs=None, tunes=None):
    """The flat peer programs under launch skew (a random 0-300 us spin ahead of every call, per
    rank): mem_2D in its three forms (launches, k_peer_oneshot, k_peer_mem_ll) and the scheduled
    BO / LO programs (k_peer_sched, its push form, k_peer_lo_ll), 6 calls of each back to back
    with no host sync, every result bit-exact vs the oracle — window parities, epochs and flag
    values must hold while the processes run out of step."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import tenstorrentallreduce_amd as t
        import oracle
        import bench
        import test_dist_host as tdh
        devs, dev, shared = placement(rank, world, devs, tunes)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        side, total = tdh.GRIDS[world]
        n = 8 * total * 16 * 12
        peer = t.Peer(world, rank, devs[rank], 4 * n)
        handles = [None] * world
        dist.all_gather_object(handles, peer.handle())
        peer.connect(handles)
        peer.set_max_groups(256 // world if shared else 0)
        s = torch.cuda.current_stream()
        cyc = bench.spin_cycles_per_us(s)
        rng = np.random.default_rng(777 + rank)
        fails = []
        # (name, knobs, program: None = mem_2D through allred_peer_allreduce, else (variant, algo))
        forms = [("mem_launches", dict(oneshot=0, mem_ll=0), None), ("mem_oneshot", dict(oneshot=1 << 40, mem_ll=0), None),
                 ("mem_ll", dict(oneshot=0, mem_ll=1 << 40), None),
                 ("bo_sched", dict(lo_ll=0, push=0), ("bo", t.SWING)), ("bo_push", dict(lo_ll=0, push=1), ("bo", t.SWING)),
                 ("lo_ll", dict(lo_ll=256 << 10, push=0), ("lo", t.RECDUB)), ("lo_sched", dict(lo_ll=0, push=0), ("lo", t.SWING))]
        for fi, (name, knobs, prog) in enumerate(forms):
            peer.set_oneshot_max(knobs.get("oneshot", 4 << 20))
            peer.set_mem_ll_max(knobs.get("mem_ll", 256 << 10))
            peer.set_lo_ll_max(knobs.get("lo_ll", 256 << 10))
            peer.set_sched_push(knobs.get("push", 0))
            calls = []
            torch.cuda.synchronize()
            dist.barrier()
            for c in range(6):
                data = tdh.inputs(world, 1, n, seed=90000 + 1000 * fi + 10 * c)
                buf = torch.from_numpy(data[rank][0].view(np.int16)).to(dev)
                torch.cuda._sleep(int(rng.integers(0, 300) * cyc))
                if prog is None:
                    peer.allreduce(buf.data_ptr(), n, s)
                else:
                    variant, algo = prog
                    desc = t.dist_desc(algo, t.BO if variant == "bo" else t.LO, side, total, n)
                    peer.dist_allreduce(desc, buf.data_ptr(), None, s)
                calls.append((data, buf))
            torch.cuda.synchronize()
            for c, (data, buf) in enumerate(calls):
                if prog is None:
                    want = [d[0].copy() for d in data]
                    oracle.allreduce("mem", 0, 1, want, world)
                    want = want[rank]
                else:
                    want = tdh.expected(prog[0], prog[1], world, 1, data, 1)[rank][0]
                bad = int((buf.cpu().numpy().view(np.uint16) != want).sum())
                if bad:
                    fails.append((name, c, bad))
        status = peer.status()
        dist.barrier()
        peer.close()
        dist.destroy_process_group()
        q.put((rank, fails, status))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())], -1))


@FENCES
@pytest.mark.parametrize("world", [2, 4, 8])
def test_peer_flat_programs_under_launch_skew_one_gpu(world, tunes):
    run_world(skew_flat_worker, world, 300, tunes=tunes)


def big_window_worker(rank, world, port, q):
    """allred_peer_create / connect with the bench's windows (1 GiB buckets,
    2 parities): an IPC-exported allocation of ~2 GiB hung in the peer's
    hipIpcOpenMemHandle on these boxes, so each parity is its own allocation.
    One small allreduce afterwards proves the mapping is live."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, ROOT)
        import tenstorrentallreduce_amd as t
        dist.init_process_group("gloo", rank=rank, world_size=world)
        peer = t.Peer(world, rank, 0, (1 << 30) // 2)
        handles = [None] * world
        dist.all_gather_object(handles, peer.handle())
        peer.connect(handles)
        fails = []
        for call in range(2):   # both parities
            buf = torch.full((8 * world * 64,), rank + 1, dtype=torch.bfloat16, device="cuda:0").view(torch.int16)
            peer.allreduce(buf.data_ptr(), buf.numel(), torch.cuda.current_stream())
            torch.cuda.synchronize()
            want = float(world * (world + 1) // 2)
            got = buf.view(torch.bfloat16).float()
            if not bool((got == want).all()):
                fails.append((call, got[:4].tolist(), want))
            dist.barrier()
        status = peer.status()
        peer.close()
        dist.destroy_process_group()
        q.put((rank, fails, status))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())], -1))


def test_peer_one_gib_windows_open_and_reduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    world = 2
    procs = [ctx.Process(target=big_window_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = []
    try:
        for _ in procs:
            results.append(q.get(timeout=90))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, fails, status in results:
        assert fails == [], (rank, fails)
        assert status & t_timeout_bit() == 0, (rank, status)


def t_timeout_bit():
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    return t.PEER_TIMEOUT


@pytest.mark.parametrize("n,cap", [(327680, 0), (327680, 7), (256 * 5, 0), (256 * 40, 3)])
def test_hier_forms_single_gpu_bit_exact(n, cap):
    """One GPU (W = 1), 64 local ranks: the one-launch form k_hier_ws (quarter / half /
    whole tiles per reducing wave) and the launch form (mem_2D exchange as one kernel or
    as launches) give the same
    bits as the oracle (tree of local rank 0 of the 8x8 Swing grid, then the
    mem_2D owner-first fp32 sum — one rank: the partial itself), twice in a row
    (both LL parities).  Config-2 size full grid and with capped grids (many
    tiles per workgroup)."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import tenstorrentallreduce_amd as t
    import oracle
    local = 64
    peer = t.Peer(1, 0, 0, 2 * n)
    peer.connect([peer.handle()])
    try:
        peer.set_max_groups(cap)
        cases = []
        for rep in range(2):
            data = np.random.default_rng(900 + rep).integers(0x3F80, 0x42C8, (local, n)).astype(np.uint16)
            loc = [x.copy() for x in data]
            oracle.allreduce("lo", 1, 8, loc, local)   # tree of local rank 0
            cases.append((data, loc[0]))
        ws = torch.empty(n, dtype=torch.int16, device="cuda:0")
        # (hier_ll, oneshot limit, k_hier_ws columns per reducing wave)
        for ll, limit, cols in ((1, 0, 16), (0, 1 << 40, 8), (1, 0, 8), (1, 0, 16), (1, 0, 32), (0, 0, 8),
                                (1, 0, 16), (1, 0, 32), (0, 1 << 40, 8), (1, 0, 8)):
            peer.set_hier_ll(ll)
            peer.set_oneshot_max(limit)
            bufs = [torch.from_numpy(d.view(np.int16)).to("cuda:0") for d, _ in cases]
            torch.cuda.synchronize()
            with t.tuned(hier_ws_cols=cols):
                for b in bufs:   # back to back: both LL parities / epochs
                    peer.allreduce(b.data_ptr(), n, torch.cuda.current_stream(), local, 8, t.SWING, ws.data_ptr())
            torch.cuda.synchronize()
            for rep, (b, (_, want)) in enumerate(zip(bufs, cases)):
                bad = int((b.cpu().numpy().view(np.uint16) != want[None, :]).sum())
                assert bad == 0, (ll, limit, cols, rep, bad)
        assert peer.status() & t.PEER_TIMEOUT == 0
    finally:
        peer.set_hier_ll(0)
        peer.close()


def test_peer_knob_argument_errors():
    """The peer knobs reject what they cannot honour (ALLRED_ERR_ARG), like the
    rest of the C-ABI; a one-rank peer set needs no second process."""
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    from tenstorrentallreduce_amd import _lib
    peer = t.Peer(1, 0, 0, 1 << 16)
    peer.connect([peer.handle()])
    try:
        with pytest.raises(_lib.AllredError):
            peer.set_hier_ll(2)            # 0 the launch form, 1 k_hier_ws (ABI 7: 2 retired with k_hier_ll)
        with pytest.raises(_lib.AllredError):
            peer.set_hier_ll(-1)
        peer.set_lo_ll_max(0)
        peer.set_mem_ll_max(0)
        peer.set_max_groups(0)
        buf = torch.zeros(1 << 17, dtype=torch.int16, device="cuda:0")
        with pytest.raises(_lib.AllredError):   # larger than the windows
            peer.allreduce(buf.data_ptr(), 1 << 17, torch.cuda.current_stream())
        with pytest.raises(_lib.AllredError):   # not a multiple of 8 elements per rank
            peer.allreduce(buf.data_ptr(), 12, torch.cuda.current_stream())
    finally:
        peer.close()


def test_peer_timeout_is_cleared():
    """A partner that never arrives: rank 0 of an in-process two-peer set
    allreduces alone, its bounded wait gives up (ALLRED_PEER_TIMEOUT, sticky),
    allred_peer_clear_status clears it, and both peers then allreduce together
    correctly — the bench drops a candidate this way without poisoning the next."""
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    peers = [t.Peer(2, r, 0, 1 << 14) for r in range(2)]
    t.Peer.connect_all(peers)
    try:
        n = 1 << 12
        bufs = [torch.full((n,), 0x3F80, dtype=torch.int16, device="cuda:0") for _ in range(2)]
        s = torch.cuda.current_stream()
        peers[0].allreduce(bufs[0].data_ptr(), n, s)   # rank 1 does not come in time
        torch.cuda.synchronize()
        assert peers[0].status() & t.PEER_TIMEOUT
        peers[1].allreduce(bufs[1].data_ptr(), n, s)   # its late call (the epochs stay paired)
        torch.cuda.synchronize()
        for p in peers:
            p.clear_status()
            assert not p.status() & t.PEER_TIMEOUT
        # a fresh pair of calls (both ranks, two streams: the two kernels wait for each other)
        s1 = torch.cuda.Stream()
        vals = [torch.full((n,), v, dtype=torch.int16, device="cuda:0") for v in (0x3F80, 0x4000)]   # 1.0, 2.0
        with torch.cuda.stream(s1):
            peers[1].allreduce(vals[1].data_ptr(), n, s1)
        peers[0].allreduce(vals[0].data_ptr(), n, s)
        torch.cuda.synchronize()
        assert not (peers[0].status() | peers[1].status()) & t.PEER_TIMEOUT
        for v in vals:   # 1.0 + 2.0 = 3.0 = 0x4040
            assert int((v.cpu() != 0x4040).sum()) == 0
    finally:
        for p in peers:
            p.close()


def config35_worker(rank, world, port, q, devs=None, tunes=None):
    """BASELINE config 3 (8-rank RecDub BO, 655,360 B per rank; one channel and
    all 7 link-spreading channels) and config 5 (8-rank Swing LO at 2 / 8 / 32 /
    128 kB; LL pushes and the scheduled flag form) through
    allred_peer_dist_allreduce with 8 processes, bit-exact vs the oracle, then
    allred_peer_check (no peer wait timed out)."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import tenstorrentallreduce_amd as t
        import test_dist_host as tdh
        devs, dev, shared = placement(rank, world, devs, tunes)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        side, total = tdh.GRIDS[world]
        peer = t.Peer(world, rank, devs[rank], 327680)
        handles = [None] * world
        dist.all_gather_object(handles, peer.handle())
        peer.connect(handles)
        fails = []
        cases = [("bo", t.RECDUB, 327680, 1, 256 << 10), ("bo", t.RECDUB, 327680, 7, 256 << 10)]
        for n in (1024, 4096, 16384, 65536):
            cases += [("lo", t.SWING, n, 1, 256 << 10), ("lo", t.SWING, n, 1, 0)]
        for ci, (variant, algo, n, chans, ll_max) in enumerate(cases):
            peer.set_lo_ll_max(ll_max)
            desc = t.dist_desc(algo, t.BO if variant == "bo" else t.LO, side, total, n, channels=chans)
            for rep in range(2):   # both window parities
                data = tdh.inputs(world, 1, n, seed=7000 + 10 * ci + rep)
                buf = torch.from_numpy(data[rank][0].view(np.int16)).to(dev)
                peer.dist_allreduce(desc, buf.data_ptr(), None, torch.cuda.current_stream(), check_status=True)
                want = tdh.expected(variant, algo, world, 1, data, chans)[rank][0]
                got = buf.cpu().numpy().view(np.uint16)
                if not np.array_equal(got, want):
                    fails.append((variant, algo, n, chans, ll_max, rep, int((got != want).sum())))
            dist.barrier()
        status = peer.status()
        dist.barrier()
        peer.close()
        dist.destroy_process_group()
        q.put((rank, fails, status))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())], -1))


@FENCES
def test_config3_config5_eight_processes(tunes):
    run_world(config35_worker, 8, 240, tunes=tunes)


@pytest.mark.parametrize("n,cap,buckets", [(327680, 0, 5), (327680, 0, 1), (256 * 5, 0, 2), (256 * 40, 5, 3),
                                           (327680, 160, 4), (256 * 40, 1, 3), (327680, 64, 3), (256 * 16, 2, 3)])
def test_hier_pipelined2_single_gpu_bit_exact(n, cap, buckets):
    """One GPU (W = 1), 64 local ranks: a sequence of buckets through the
    two-deep pipelined hierarchical step (k_hier_x2: launch i starts bucket i,
    sums bucket i-1's owned tiles and writes bucket i-2), buckets + 1 calls
    (1 bucket: the flush sums and writes it; 2: the flush writes both), every
    bucket bit-exact vs the oracle; full and capped grids (one workgroup with
    40 tiles: five chunks of staged results; exactly one chunk per workgroup),
    the sequence repeated (both LL parities reused).  Protocol errors: another
    peer call while buckets are pending, a different bucket size mid-sequence, a
    flush with nothing pending."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import tenstorrentallreduce_amd as t
    from tenstorrentallreduce_amd import _lib
    import oracle
    local = 64
    peer = t.Peer(1, 0, 0, 2 * n)
    peer.connect([peer.handle()])
    try:
        peer.set_max_groups(cap)
        data, want = [], []
        for b in range(buckets):
            d = np.random.default_rng(2300 + b).integers(0x3F80, 0x42C8, (local, n)).astype(np.uint16)
            loc = [x.copy() for x in d]
            oracle.allreduce("lo", 1, 8, loc, local)   # tree of local rank 0
            data.append(torch.from_numpy(d.view(np.int16)).to("cuda:0"))
            want.append(loc[0])
        s = torch.cuda.current_stream()
        for rep in range(4):   # the sequence again and again: both parities, epochs advancing
            bufs = [x.clone() for x in data]
            for b in bufs:
                peer.allreduce_pipelined2(b.data_ptr(), n, s)
            peer.allreduce_pipelined2(None, n, s)
            torch.cuda.synchronize()
            for i, (b, w) in enumerate(zip(bufs, want)):
                bad = int((b.cpu().numpy().view(np.uint16) != w[None, :]).sum())
                assert bad == 0, (rep, i, bad)
        assert peer.status() & t.PEER_TIMEOUT == 0
        x = data[0].clone()
        peer.allreduce_pipelined2(x.data_ptr(), n, s)
        with pytest.raises(_lib.AllredError):   # another call while a bucket is pending
            peer.allreduce(x.data_ptr(), n, s, local, 8, t.SWING, x.data_ptr())
        if n % (2 * 256) == 0:
            with pytest.raises(_lib.AllredError):   # another bucket size mid-sequence
                peer.allreduce_pipelined2(x.data_ptr(), n // 2, s)
        peer.allreduce_pipelined2(None, n, s)
        with pytest.raises(_lib.AllredError):   # nothing pending
            peer.allreduce_pipelined2(None, n, s)
        torch.cuda.synchronize()
        assert (x.cpu().numpy().view(np.uint16) == want[0][None, :]).all()
        # one-launch calls right after a sequence (LL parities and epochs continue)
        peer.set_hier_ll(1)
        ys = [data[i % buckets].clone() for i in range(3)]
        ws = torch.empty(n, dtype=torch.int16, device="cuda:0")
        for y in ys:
            peer.allreduce(y.data_ptr(), n, s, local, 8, t.SWING, ws.data_ptr())
        torch.cuda.synchronize()
        for i, y in enumerate(ys):
            assert (y.cpu().numpy().view(np.uint16) == want[i % buckets][None, :]).all(), i
        assert peer.status() & t.PEER_TIMEOUT == 0
    finally:
        peer.close()


@pytest.mark.parametrize("first_tiles", [64, 32])
def test_hier_handoff_epoch_wrap_is_cleared(first_tiles):
    """The hierarchical forms' hand-off words carry a 16-bit epoch ((k + 1) %
    65535 + 1 for call k), so call k + 131070 (same parity) awaits the epoch
    call k's words carry.  A bucket of `first_tiles` tiles at call 0, then
    131069 two-tile ones, then a 64-tile bucket at call 131070: the slots beyond
    the small buckets' range still hold call 0's words with call 131070's epoch
    — also when the last bucket is LARGER than call 0's (32 -> 64 tiles: slots
    32..63 were never written, slots 2..31 hold call 0's words; advisor r05).
    The host sees it coming (hier_area_prepare) and clears the parity's area
    between two barriers; the result must be call 131070's own data, bit-exact
    (W = 1, k_hier_ws with ONE workgroup: every owned tile past its 16 LDS
    slots crosses the own inbox, so a stale word would be read).  ~2 s of tiny
    launches."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import tenstorrentallreduce_amd as t
    import oracle
    local, small, large = 64, 256 * 2, 256 * 64
    peer = t.Peer(1, 0, 0, 2 * large)
    peer.connect([peer.handle()])
    try:
        peer.set_hier_ll(1)
        peer.set_max_groups(1)
        s = torch.cuda.current_stream()
        ws = torch.empty(large, dtype=torch.int16, device="cuda:0")

        def bucket(seed, n):
            d = np.random.default_rng(seed).integers(0x3F80, 0x42C8, (local, n)).astype(np.uint16)
            loc = [x.copy() for x in d]
            oracle.allreduce("lo", 1, 8, loc, local)   # tree of local rank 0
            return torch.from_numpy(d.view(np.int16)).to("cuda:0"), loc[0]

        first, want0 = bucket(1, 256 * first_tiles)
        peer.allreduce(first.data_ptr(), 256 * first_tiles, s, local, 8, t.SWING, ws.data_ptr())    # call 0
        torch.cuda.synchronize()
        assert int((first.cpu().numpy().view(np.uint16) != want0[None, :]).sum()) == 0
        sm, _ = bucket(2, small)   # reduced in place over and over: only its launches matter
        for i in range(131069):                                                         # calls 1 .. 131069
            peer.allreduce(sm.data_ptr(), small, s, local, 8, t.SWING, ws.data_ptr())
            if i % 16384 == 16383:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        assert peer.status() & t.PEER_TIMEOUT == 0
        last, want = bucket(3, large)
        peer.allreduce(last.data_ptr(), large, s, local, 8, t.SWING, ws.data_ptr())     # call 131070
        torch.cuda.synchronize()
        bad = int((last.cpu().numpy().view(np.uint16) != want[None, :]).sum())
        assert bad == 0, bad
        assert peer.status() & t.PEER_TIMEOUT == 0
    finally:
        peer.set_hier_ll(0)
        peer.set_max_groups(0)
        peer.close()


def wrap_worker(rank, world, port, q, devs=None, tunes=None):
    """The epoch-wrap clear where a stale word would be READ: W processes, one bucket of
    `first` tiles at call 0, 131069 two-tile calls, then a bucket of 64 tiles at call 131070
    that rank W-1 joins ~3 ms late (a spin ahead of its launch).  The other ranks' writing
    waves poll their inbox slots for rank W-1's partials at once; slots that still hold call
    0's words carry call 131070's 16-bit epoch, so without the clear they are taken as this
    call's partials (wrong sums); with it every word waits for rank W-1."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import tenstorrentallreduce_amd as t
        import oracle
        import bench
        first = int(os.environ.get("WRAP_FIRST_TILES", "32"))
        devs, dev, shared = placement(rank, world, devs, tunes)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        local, small, large = 64, 256 * world, 256 * 64
        peer = t.Peer(world, rank, devs[rank], large)
        handles = [None] * world
        dist.all_gather_object(handles, peer.handle())
        peer.connect(handles)
        peer.set_max_groups(256 // world if shared else 0)
        peer.set_hier_ll(1)
        s = torch.cuda.current_stream()
        ws = torch.empty(large, dtype=torch.int16, device=dev)

        def data(c, r, n):
            return np.random.default_rng(7000 + 100 * c + r).integers(0x3F80, 0x42C8, (local, n)).astype(np.uint16)

        def expected(c, n):
            partials = []
            for r in range(world):
                loc = [x.copy() for x in data(c, r, n)]
                oracle.allreduce("lo", 1, 8, loc, local)   # tree of local rank 0
                partials.append(loc[0])
            oracle.allreduce("mem", 0, 1, partials, world)
            return partials[rank]

        fails = []
        b0 = torch.from_numpy(data(0, rank, 256 * first).view(np.int16)).to(dev)
        peer.allreduce(b0.data_ptr(), 256 * first, s, local, 8, t.SWING, ws.data_ptr())   # call 0
        sm = torch.from_numpy(data(1, rank, small).view(np.int16)).to(dev)
        for i in range(131069):                                                         # calls 1 .. 131069
            peer.allreduce(sm.data_ptr(), small, s, local, 8, t.SWING, ws.data_ptr())
            if i % 16384 == 16383:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        b2 = torch.from_numpy(data(2, rank, large).view(np.int16)).to(dev)
        torch.cuda.synchronize()
        dist.barrier()
        if rank == world - 1:
            torch.cuda._sleep(int(3000 * bench.spin_cycles_per_us(s)))
        peer.allreduce(b2.data_ptr(), large, s, local, 8, t.SWING, ws.data_ptr())     # call 131070
        torch.cuda.synchronize()
        bad = int((b2.cpu().numpy().view(np.uint16) != expected(2, large)[None, :]).sum())
        if bad:
            fails.append(("call 131070", bad))
        status = peer.status()
        dist.barrier()
        peer.set_hier_ll(0)
        peer.close()
        dist.destroy_process_group()
        q.put((rank, fails, status))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())], -1))


@pytest.mark.parametrize("first_tiles", [64, 32])
def test_hier_handoff_epoch_wrap_across_processes(first_tiles, monkeypatch):
    """tests the clear where a late peer makes a stale word readable (2 processes, rank 1 late)."""
    monkeypatch.setenv("WRAP_FIRST_TILES", str(first_tiles))
    run_world(wrap_worker, 2, 300)

