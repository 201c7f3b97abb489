"""The N > 1 paths across REAL devices, bit-exact against the oracle whenever
more than one GPU is visible.

Every other GPU test runs the multi-GPU code on one device (a 1-rank RCCL
communicator, or G peer processes / threads sharing the card).  Here each
case needs G visible GPUs and skips with that reason otherwise (the driver's
1-GPU box), so the first multi-GPU box turns the suite into parity evidence
for what the 8-GPU node runs — the reference validates every run
(allred_helper.hpp:84-96 -> validate_result_vector, allred_helper.cpp:18-120):
- the reference executables with ALLRED_GPUS=G over RCCL and over the peer
  windows, one group per device (no ALLRED_SHARE_GPU): "All values match!" at
  ERROR 0 for every INTEGRATION.md §1 invocation, and the oracle's
  composition of the plan on arbitrary data;
- the RCCL programs (allred_dist_allreduce, one thread per device on
  allred_comm_init_all communicators): BO / LO / mem_2D x Swing / RecDub / 1D,
  flat and hierarchical, the link-spreading channels on a >= 1 MiB bucket, the
  pipelined form (rccl_x) with 64 local ranks;
- the peer windows across devices (IPC-mapped, one process per GPU: the
  bench's path): every scheduled / pushed / LL / hierarchical form of
  tests/test_gpu_peer.py's workers, also with tune peer_fence=1 (a release
  fence before every flag or LL hand-off store, an acquire fence after every
  wait: the same bits);
- BASELINE config 4 (8-rank Swing BO, 1 GiB per GPU; at G = 2 / 4 on the
  smaller grids) by exact sums of small integers (every reduction order is
  exact), over RCCL and the peer windows (pull and push forms).
ALLRED_TEST_REHEARSE=1 runs the peer-window cases with every rank on device 0
(the harness itself rehearsed on a 1-GPU box); the RCCL cases still skip
(RCCL refuses two ranks on one device)."""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

import tenstorrentallreduce_amd as t
import test_dist_host as tdh
import test_gpu_peer as tgp
import multi_cases as mc
from multi_cases import BIN, argv_error0, expected, invocations

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
NG = torch.cuda.device_count()   # counts devices without initialising HIP
REHEARSE = os.environ.get("ALLRED_TEST_REHEARSE") == "1"
WORLDS = (2, 4, 8)
FENCES = ({}, {"peer_fence": 1})


def devices(g, peer=True):
    """Device of each of g ranks: one GPU each; the rehearsal puts peer ranks on device 0."""
    if NG >= g:
        return list(range(g))
    if REHEARSE and peer and NG >= 1:
        return [0] * g
    pytest.skip(f"needs {g} GPUs, {NG} visible" + ("" if peer else " (RCCL: one rank per device)"))


# ---------------------------------------------------------------- the executables across GPUs
CLI_CASES = [(tr, g, *inv) for tr in ("rccl", "peer") for g in WORLDS for inv in invocations(g)]
CLI_IDS = [f"{c[0]}-g{c[1]}-{c[2]}" for c in CLI_CASES]


def _cli_env(transport, g, nodes):
    devs = devices(g, peer=transport == "peer")
    e = dict(os.environ)
    e.update({"ALLRED_TRANSPORT": transport, "ALLRED_GPUS": str(g), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
              "ALLRED_SHARE_GPU": "1" if len(set(devs)) < g else "0"})
    if len(set(devs)) < g:   # the rehearsal: every group's stream on a hardware queue of its own
        e["GPU_MAX_HW_QUEUES"] = "16"
    e.pop("ALLRED_NODES", None)
    if nodes is not None:
        e["ALLRED_NODES"] = str(nodes)
    return e


@pytest.mark.parametrize("transport,g,name,variant,argv,nodes", CLI_CASES, ids=CLI_IDS)
def test_cli_across_gpus(transport, g, name, variant, argv, nodes):
    """The reference executable with ALLRED_GPUS=G, group g on device g: "All
    values match!" at ERROR 0 (RNE ctor), every rank validated, strict exit."""
    env = _cli_env(transport, g, nodes)
    env.update({"ALLRED_CHECK_ALL": "1", "ALLRED_BF16_ROUND": "rne", "ALLRED_STRICT": "1", "ALLRED_REPORT": "1"})
    r = subprocess.run([os.path.join(t._lib.BIN_DIR, BIN[variant]), *argv_error0(argv, variant)],
                       capture_output=True, text=True, env=env, timeout=180)
    assert r.returncode == 0, (r.stdout, r.stderr[-3000:])
    assert r.stdout.strip() == "All values match!", r.stdout
    assert '"mismatches": 0' in r.stderr


@pytest.mark.parametrize("transport,g,name,variant,argv,nodes", CLI_CASES, ids=CLI_IDS)
def test_cli_across_gpus_bit_exact_vs_oracle(tmp_path, transport, g, name, variant, argv, nodes):
    """Arbitrary per-rank data through allred_run_multi across G devices: every
    rank equals the oracle's composition of the plan bit for bit."""
    env = _cli_env(transport, g, nodes)
    out = tmp_path / "out.npy"
    seed = 131 * g + len(name) + (7 if transport == "rccl" else 0)
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_multi_child.py"), str(variant), str(g),
                        "-" if nodes is None else str(nodes), str(seed), str(out), "--", *argv],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, (r.stdout, r.stderr[-3000:])
    data, got = np.load(out)
    old = os.environ.get("ALLRED_NODES")
    try:
        os.environ.pop("ALLRED_NODES", None)
        if nodes is not None:
            os.environ["ALLRED_NODES"] = str(nodes)
        plan = t.multi_plan(["x", *argv], variant, gpus=g)
    finally:
        os.environ.pop("ALLRED_NODES", None)
        if old is not None:
            os.environ["ALLRED_NODES"] = old
    bad = int((got != expected(plan, data)).sum())
    assert bad == 0, f"{transport} {name} G={g}: {bad} elements differ"


# ---------------------------------------------------------------- RCCL programs, one thread per device
def _threads(world, fn):
    errs = []

    def one(g):
        try:
            torch.cuda.set_device(g)
            fn(g)
        except Exception as e:  # reported below
            import traceback
            errs.append((g, repr(e), traceback.format_exc()[-1500:]))

    th = [threading.Thread(target=one, args=(g,)) for g in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not any(x.is_alive() for x in th), "an RCCL thread never returned"
    assert not errs, errs


@pytest.mark.parametrize("world", WORLDS)
def test_rccl_programs_across_gpus(world):
    """allred_dist_allreduce over real RCCL communicators (allred_comm_init_all,
    one thread per device): every case of tests/test_dist_host.py's gloo matrix,
    the auto channels on a 1 MiB bucket and mem_2D (fp32 and the reference's
    bf16 accumulation), each twice back to back, bit-exact vs the oracle.  The
    cases and the expected values are tests/multi_cases.py's, run on CPU through
    the host twin of the same program by tests/test_multidevice_host.py."""
    devs = devices(world, peer=False)
    side, total = tdh.GRIDS[world]
    torch.cuda.set_device(0)
    comms = t.Comm.init_all(devs)
    try:
        torch.cuda.synchronize(0)
        assert torch.cuda.current_device() == 0   # init_all leaves the caller's device alone (advisor r04)
        for ci, (variant, algo, local, chans, n) in enumerate(mc.rccl_cases(world)):
            desc = mc.rccl_case_desc(world, variant, algo, local, chans, n)
            runs = [mc.rccl_case_inputs(world, local, n, ci, rep) for rep in range(2)]
            got = [[None] * world for _ in runs]

            def step(g):
                s = torch.cuda.current_stream(g)
                ws = torch.empty(max(t.dist_workspace_bytes(desc), 16), dtype=torch.uint8, device=f"cuda:{g}")
                bufs = [torch.from_numpy(np.concatenate(data[g]).view(np.int16)).to(f"cuda:{g}") for data in runs]
                for b in bufs:
                    t.dist_allreduce(comms[g], desc, b.data_ptr(), ws.data_ptr(), s)
                comms[g].wait(s)
                for k, b in enumerate(bufs):
                    got[k][g] = b.cpu().numpy().view(np.uint16)

            _threads(world, step)
            for k, data in enumerate(runs):
                want = mc.rccl_case_expected(world, variant, algo, local, chans, n, data)
                for g in range(world):
                    assert np.array_equal(got[k][g], want[g]), (variant, algo, local, chans, n, k, g)
        for acc in (t.ACC_FP32, t.ACC_BF16):
            n = 8 * total * 640
            desc = t.dist_desc(t.SWING, t.MEM, side, total, n, mem_accum=acc)
            data = mc.rccl_mem_inputs(world, acc, n)
            got = [None] * world

            def mem(g):
                s = torch.cuda.current_stream(g)
                ws = torch.empty(t.dist_workspace_bytes(desc), dtype=torch.uint8, device=f"cuda:{g}")
                b = torch.from_numpy(data[g].view(np.int16)).to(f"cuda:{g}")
                t.dist_allreduce(comms[g], desc, b.data_ptr(), ws.data_ptr(), s)
                comms[g].wait(s)
                got[g] = b.cpu().numpy().view(np.uint16)

            _threads(world, mem)
            want = mc.rccl_mem_expected(world, acc, data)
            for g in range(world):
                assert np.array_equal(got[g], want[g]), ("mem", acc, g)
    finally:
        for c in comms:
            c.close()


@pytest.mark.parametrize("world", WORLDS)
def test_rccl_pipelined_across_gpus(world):
    """allred_dist_allreduce_pipelined (the rccl_x transport) with 64 local
    ranks per device at config-2 size: K buckets in K + 1 calls, every bucket
    = the oracle's tree of local rank 0 (8x8 Swing), then the 2D Swing BO of
    the partials over the GPU grid (link-spreading channels where the bucket
    takes them), written to all 64 rows."""
    devs = devices(world, peer=False)
    side, total = tdh.GRIDS[world]
    n, local, K = 327680, 64, 3
    desc = t.dist_desc(t.SWING, t.BO, side, total, n, local_ranks=local, local_side=8, local_algo=t.SWING)
    data = mc.pipelined_inputs(world, n, local, K)
    comms = t.Comm.init_all(devs)
    got = [[None] * world for _ in range(K)]
    try:
        def step(g):
            s = torch.cuda.current_stream(g)
            ws = torch.empty(2 * t.dist_workspace_bytes(desc), dtype=torch.uint8, device=f"cuda:{g}")
            bufs = [torch.from_numpy(d[g].view(np.int16)).to(f"cuda:{g}") for d in data]
            for b in bufs:
                t.dist_allreduce_pipelined(comms[g], desc, b.data_ptr(), ws.data_ptr(), s)
            t.dist_allreduce_pipelined(comms[g], desc, None, ws.data_ptr(), s)
            comms[g].wait(s)
            for k, b in enumerate(bufs):
                got[k][g] = b.cpu().numpy().view(np.uint16)

        _threads(world, step)
    finally:
        for c in comms:
            c.close()
    for k in range(K):
        partials = mc.pipelined_expected(world, n, data[k], local)
        for g in range(world):
            bad = int((got[k][g] != partials[g][None, :]).sum())
            assert bad == 0, (k, g, bad)


# ---------------------------------------------------------------- peer windows across devices
@pytest.mark.parametrize("tunes", FENCES, ids=["relaxed", "fenced"])
@pytest.mark.parametrize("world", WORLDS)
def test_peer_mem_and_hier_forms_across_gpus(world, tunes):
    """tests/test_gpu_peer.py's worker with one process per device: mem_2D
    (launches, k_peer_oneshot, k_peer_mem_ll), the hierarchical forms (k_hier_ws
    over quarter / half / whole tiles, the launch form, k_hier_x2, capped grids)."""
    tgp.run_world(tgp.worker, world, 300, devs=devices(world), tunes=tunes)


@pytest.mark.parametrize("tunes", FENCES, ids=["relaxed", "fenced"])
@pytest.mark.parametrize("world", WORLDS)
def test_peer_scheduled_programs_across_gpus(world, tunes):
    """tests/test_gpu_peer.py's dist_worker with one process per device: the
    Swing / RecDub / 1D BO and LO programs over the peer windows (k_peer_sched,
    k_peer_sched_push, k_peer_lo_ll), flat and hierarchical, channels."""
    tgp.run_world(tgp.dist_worker, world, 300, devs=devices(world), tunes=tunes)


@pytest.mark.parametrize("world", WORLDS)
def test_peer_hier_handoffs_under_launch_skew_across_gpus(world):
    """tests/test_gpu_peer.py's skew_worker with one process per device: k_hier_ws calls and a
    k_hier_x2 sequence with random spins (0-300 us) ahead of every call, bit-exact."""
    tgp.run_world(tgp.skew_worker, world, 300, devs=devices(world))


@pytest.mark.parametrize("first_tiles", [64, 32])
def test_peer_hier_epoch_wrap_across_gpus(first_tiles, monkeypatch):
    """tests/test_gpu_peer.py's wrap_worker with one process per device: the hand-off area's
    epoch-wrap clear where a late peer makes a stale word readable, bit-exact."""
    monkeypatch.setenv("WRAP_FIRST_TILES", str(first_tiles))
    tgp.run_world(tgp.wrap_worker, 2, 300, devs=devices(2))


@pytest.mark.parametrize("tunes", FENCES, ids=["relaxed", "fenced"])
@pytest.mark.parametrize("world", WORLDS)
def test_peer_flat_programs_under_launch_skew_across_gpus(world, tunes):
    """tests/test_gpu_peer.py's skew_flat_worker with one process per device: mem_2D (launches,
    one-shot, LL) and the scheduled BO / LO programs (pull, push, LL) with random spins ahead of
    every call, bit-exact."""
    tgp.run_world(tgp.skew_flat_worker, world, 300, devs=devices(world), tunes=tunes)


@pytest.mark.parametrize("tunes", FENCES, ids=["relaxed", "fenced"])
def test_peer_config3_config5_across_8_gpus(tunes):
    """BASELINE configs 3 and 5 over the peer windows with one process per device."""
    tgp.run_world(tgp.config35_worker, 8, 300, devs=devices(8), tunes=tunes)


# ---------------------------------------------------------------- config 4: 1 GiB per GPU
GIB_ELEMS = 1 << 29   # 1 GiB of bf16 per GPU


_ints = mc.config4_ints     # rank r's bucket: small integers 0..7 in bf16, exact sums in any order
_exact = mc.config4_exact


@pytest.mark.parametrize("world", WORLDS)
def test_config4_one_gib_over_rccl_across_gpus(world):
    """BASELINE config 4 (Swing BO, 1 GiB per GPU, every link: auto channels)
    over RCCL: every GPU's bucket equals the exact sum of the ranks' buckets."""
    devs = devices(world, peer=False)
    side, total = tdh.GRIDS[world]
    desc = t.dist_desc(t.SWING, t.BO, side, total, GIB_ELEMS)
    comms = t.Comm.init_all(devs)
    bad = [None] * world
    try:
        def step(g):
            dev = f"cuda:{g}"
            s = torch.cuda.current_stream(g)
            b = _ints(GIB_ELEMS, g, dev)
            ws = torch.empty(t.dist_workspace_bytes(desc), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(g)
            t.dist_allreduce(comms[g], desc, b.data_ptr(), ws.data_ptr(), s)
            comms[g].wait(s)
            bad[g] = int((b.float() != _exact(GIB_ELEMS, world, dev)).sum())

        _threads(world, step)
    finally:
        for c in comms:
            c.close()
    assert bad == [0] * world, bad


def config4_peer_worker(rank, world, port, q, devs=None, tunes=None):
    """Config 4 over the peer windows, one process per GPU: the pulled (k_peer_sched)
    and pushed (k_peer_sched_push) forms, auto channels, exact sums."""
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, os.path.dirname(HERE))
        import tenstorrentallreduce_amd as t
        devs, dev, shared = tgp.placement(rank, world, devs, tunes)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        side, total = tdh.GRIDS[world]
        peer = t.Peer(world, rank, devs[rank], GIB_ELEMS)
        handles = [None] * world
        dist.all_gather_object(handles, peer.handle())
        peer.connect(handles)
        if shared:
            peer.set_max_groups(256 // world)
        desc = t.dist_desc(t.SWING, t.BO, side, total, GIB_ELEMS)
        fails = []
        want = _exact(GIB_ELEMS, world, dev)
        for push in (0, 1):
            peer.set_sched_push(push)
            b = _ints(GIB_ELEMS, rank, dev)
            torch.cuda.synchronize()
            dist.barrier()
            peer.dist_allreduce(desc, b.data_ptr(), None, torch.cuda.current_stream(), check_status=True)
            nbad = int((b.float() != want).sum())
            if nbad:
                fails.append(("push" if push else "pull", nbad))
            dist.barrier()
        status = peer.status()
        peer.close()
        dist.destroy_process_group()
        q.put((rank, fails, status))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())], -1))


@pytest.mark.parametrize("world", WORLDS)
def test_config4_one_gib_over_peer_windows_across_gpus(world):
    tgp.run_world(config4_peer_worker, world, 300, devs=devices(world))
