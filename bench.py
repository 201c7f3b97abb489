#!/usr/bin/env python3
"""bench.py — allreduce GB/s of the MI355X engine (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N ... bench.py --gpus N --steps K --warmup W

A step is one allreduce of device-resident bf16 buckets:
  N = 1  BASELINE config 2: the 8x8 Swing BO allreduce of 64 virtual ranks x
         655,360 B (5 tiles per block) in one MI355X's HBM, executed as the
         one-pass fused HIP kernel (k_tree_lds_lag<64>, bit-exact with the
         12-step schedule).  32 rotating bucket sets (1.3 GB, 5x the 256 MiB Infinity
         Cache) so every step streams from HBM; K < 100 steps are eager launches
         behind a spin kernel, K >= 100 replays of a captured HIP graph
         (DESIGN.md §6); ms_per_step = the median of 5 repetitions / K.
         Beside it: the tile-sum (k_add) at 256 MiB and 1 GiB with its own roofline.
  N > 1  weak scaling: every GPU holds its own 64 x 640 kB ranks (same set
         rotation); on-GPU tree reduce -> 2D Swing BO between the N GPUs (grid
         (2,2), (2,4), (4,8)) over RCCL/xGMI or peer-mapped windows, or the
         one-kernel hierarchical form -> back to the 64 ranks; the transport
         is the fastest one verified on the machine running it (exact sums and
         the reference's closed form, verify_transport), median of 3
         repetitions; every xGMI arm (configs 3-5) is verified before it is
         timed, and the CPU loopback of configs 3-5 is timed beside it.
value = bytes of all ranks' buckets allreduced per second, whole job (GB/s, 1e9).
Rank 0 prints ONE JSON line.  See DESIGN.md §Measurement for every field.
"""
from __future__ import annotations

import time

_T0 = time.perf_counter()   # the N > 1 budget counts from here (imports included: the driver's clock does)

import argparse  # noqa: E402
import contextlib  # noqa: E402
import json
import os  # noqa: E402
import statistics  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402
import threading  # noqa: E402
import traceback  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (plumbing: device memory, streams, events, gloo)
import torch.distributed as dist  # noqa: E402

import tenstorrentallreduce_amd as t  # noqa: E402

HBM_PEAK_GBPS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
METRIC = "allreduce GB/s (device-resident bf16 buckets) at 1/2/4/8 MI355X; % xGMI peak"   # BASELINE.json
XGMI_LINK_DIR_GBPS = 76.8     # 153.6 GB/s per link quoted bidirectional -> per direction
SIDE, RANKS, TILES = 8, 64, 5
ELEMS = t.normalize_tiles(TILES, RANKS, True) * 1024   # 327,680 bf16 = 655,360 B per rank
GRIDS = {1: (1, 1), 2: (2, 2), 4: (2, 4), 8: (4, 8)}


def cpu_cores() -> int:
    n = len(os.sched_getaffinity(0))
    try:  # cgroup v2 quota (the GPU box shares its CPUs: 16 per GPU)
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except Exception:
        pass
    return n


def fill_reference_convention(buf: torch.Tensor, seed: int) -> None:
    """Synthetic inputs of the reference's shape: uniform [0,100) bf16, even-x
    ranks get src_1, odd-x ranks src_0 (allred_BO_2D.cpp:79-85)."""
    g = torch.Generator(device=buf.device).manual_seed(seed)
    n = buf.shape[1]
    a = (torch.rand(n, generator=g, device=buf.device) * 100).to(torch.bfloat16).view(torch.int16)
    b = (torch.rand(n, generator=g, device=buf.device) * 100).to(torch.bfloat16).view(torch.int16)
    for r in range(buf.shape[0]):
        buf[r].copy_(b if (r % SIDE) % 2 == 0 else a)


def cpu_baseline() -> dict:
    """The oracle's loopback multi-process restatement (oracle/allred_oracle_cli)
    on this host's cores: same config 2 allreduce, ~10 s of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    argv = [1, 1, SIDE, 13, TILES, 32, 0, 1]
    probe = oracle.loopback("bo", argv, reps=3)
    reps = int(min(400, max(5, 10.0 / max(probe["median_s"], 1e-4))))
    log = os.path.join(ROOT, "gpurun_out", "cpu_baseline_profile_log.csv")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    out = oracle.loopback("bo", argv, reps=reps, timeout=300, profile_log=log)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from profile_analyzer import analyze  # profiler_results_analyzer.py statistics over the 64 ranks
    secs = out["seconds"]
    median_rep = sorted(range(len(secs)), key=lambda i: secs[i])[len(secs) // 2]
    per_rank = analyze(log, run_id=median_rep)   # the rep of median time (one slow rep says nothing)
    bytes_all = RANKS * ELEMS * 2
    # BASELINE config 1 on the CPU: the reference's own CPU-runnable case
    # (allred_BO_2D 0 1 2 -1 1 32 0 0: 2x2 RecDub LO, 1 tile, all ones), 4 rank processes
    c1 = oracle.loopback("bo", [0, 1, 2, -1, 1, 32, 0, 0], reps=200, timeout=120)
    return {
        "value": round(bytes_all / out["median_s"] / 1e9, 4),
        "unit": "GB/s",
        "cores": min(RANKS, cpu_cores()),
        "kind": "port",
        "sample": (f"oracle loopback (64 forked rank processes, shared-memory buffers, semaphore handshakes) "
                   f"of the full config-2 allreduce, {reps} reps, median {out['median_s'] * 1e3:.3f} ms "
                   f"(min {out['min_s'] * 1e3:.3f}, max {out['max_s'] * 1e3:.3f}); mismatches {out['mismatches']}"),
        "online_cpus": os.sysconf("SC_NPROCESSORS_ONLN"),
        "per_rank_median_rep_ns": per_rank,
        "config1": {"us_per_allreduce_median": round(c1["median_s"] * 1e6, 3), "cores": min(4, cpu_cores()),
                    "sample": f"oracle loopback, 4 rank processes, 200 reps; mismatches {c1['mismatches']}"},
    }


# the fused BO kernel the engine launches at config 2 (kernels.hip launch_tree_fused)
FUSED_KERNEL = "k_tree_lds_lag<64>"


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed PMC summary
    (tools/pmc_traffic.py: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc
    passes of bench.py --main-only, gfx950 FETCH_SIZE x2 correction), only when
    that summary was taken on the same kernel template this bench launches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        e = d["kernels"][kernel]
        return e["hbm_bytes_per_launch"] if e.get("template") == kernel else None
    except Exception:
        return None


def tilesum(stream, steps: int, reps: int, sizes=(256 << 20, 1 << 30)) -> dict:
    """The local tile-sum (north_star: >= 70 % of per-GPU HBM peak): dst += src
    in bf16 through allred_bf16_add (k_add, the per-step add of
    allred_BO_2D/kernels/compute_kernel.cpp:53-60 over a whole bucket) at 256 MiB
    and 1 GiB.  Checked once against the torch fp32 reference of the same op
    (fp32 add, RNE to bf16), then timed: R repetitions of K back-to-back adds,
    median; algorithmic bytes 3 * n * 2 (two reads, one write) per launch."""
    out = {}
    for nbytes in sizes:
        n = nbytes // 2
        g = torch.Generator(device="cuda:0").manual_seed(nbytes & 0xFFFF)
        dst = (torch.rand(n, generator=g, device="cuda:0") * 100).to(torch.bfloat16)
        src = (torch.rand(n, generator=g, device="cuda:0") * 100).to(torch.bfloat16)
        want = (dst.float() + src.float()).to(torch.bfloat16)
        torch.cuda.synchronize()
        t.bf16_add(dst.data_ptr(), src.data_ptr(), n, stream)
        torch.cuda.synchronize()
        ok = torch.equal(dst.view(torch.int16), want.view(torch.int16))
        del want
        k = max(5, min(steps, 50))
        with torch.cuda.stream(stream):
            for _ in range(3):
                t.bf16_add(dst.data_ptr(), src.data_ptr(), n, stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        torch.cuda.synchronize()
        ev[0].record(stream)
        for r in range(reps):
            for _ in range(k):
                t.bf16_add(dst.data_ptr(), src.data_ptr(), n, stream)
            ev[r + 1].record(stream)
        torch.cuda.synchronize()
        ms = statistics.median(ev[r].elapsed_time(ev[r + 1]) for r in range(reps)) / k
        alg = 3 * nbytes
        ach = alg / (ms * 1e-3) / 1e9
        out[f"{nbytes >> 20}MiB"] = {
            "ms_per_add": round(ms, 5), "matches_torch_fp32": ok, "adds_per_repetition": k, "repetitions": reps,
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": pmc_traffic(f"k_add@{nbytes >> 20}MiB"),
                         "kernel": "k_add", "algorithmic_bytes_per_launch": alg}}
        del dst, src
    return out


def bench_single(args) -> dict:
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(device=dev)
    nsets = args.sets
    stride = t.preferred_rank_stride(ELEMS)   # 128-byte skew between rank rows
    sets = [torch.empty((RANKS, stride), dtype=torch.int16, device=dev) for _ in range(nsets)]
    for i, s in enumerate(sets):
        fill_reference_convention(s[:, :ELEMS], 1000 + i)
    torch.cuda.synchronize()
    plan = t.Plan(t.SWING, t.BO, SIDE, ELEMS, RANKS, t.EXEC_FUSED)
    steps_plan = t.Plan(t.SWING, t.BO, SIDE, ELEMS, RANKS, t.EXEC_STEPS)

    def step(i, p=plan):
        p.execute(sets[i % nsets].data_ptr(), stride, None, stream)

    # How the K timed steps are issued (tools/timing_probe.py, profiles/r02_timing_methods.jsonl):
    #   K >= 100: R back-to-back replays of a K-step HIP graph; each replay of a
    #     ROCm graph starts with a fixed ~7 us of GPU-side launch latency, which
    #     costs < 0.1 us per step here (K = 200: 14.02 us graph vs 14.14 eager);
    #   K < 100: K eager launches behind a spin kernel that covers the host's
    #     submission (K = 20: 14.2-14.4 us vs 14.4-14.6 for graph replays).
    # The graph is captured BEFORE the prewarm, so no host-only phase sits
    # between the steady-clock prewarm and the timed steps.
    use_graph = not args.eager and args.steps >= 100
    graph = None
    if use_graph:
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                for i in range(args.steps):
                    step(i)
            torch.cuda.synchronize()
        except Exception as e:  # fall back to eager launches, say so
            print(f"[bench] graph capture failed ({e}); eager launches", file=sys.stderr)
            graph = None

    def k_steps():   # one pass over the K timed steps
        with torch.cuda.stream(stream):
            if graph is not None:
                graph.replay()
            else:
                for i in range(args.steps):
                    step(i)

    with torch.cuda.stream(stream):
        prewarm_s = prewarm(lambda i: k_steps() if graph is not None else step(i), args.prewarm_ms,
                            batch=max(1, 200 // args.steps) if graph is not None else 50)
        for i in range(args.warmup):
            step(i)
    torch.cuda.synchronize()

    # R repetitions of the K timed steps, an event between consecutive ones;
    # ms_per_step = the median repetition / K (each interval is exactly K
    # steps).  The whole R x K region is bracketed by synchronize on both sides.
    reps = max(1, args.reps)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        # a spin kernel ahead of the first event keeps the GPU busy while the host
        # submits (eager: ~4 us of host time per launch; host_wall_s below includes everything)
        torch.cuda._sleep(max(200000, 15000 * args.steps * (1 if graph is not None else reps)))
    ev[0].record(stream)
    for r in range(reps):
        k_steps()
        ev[r + 1].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    rep_ms = [ev[r].elapsed_time(ev[r + 1]) for r in range(reps)]
    ms_per_step = statistics.median(rep_ms) / args.steps
    e0, e1 = ev[0], ev[1]
    fused_launch = t.last_launch()   # the bench kernel's grid and residency (launched in the warmup)

    bytes_all = RANKS * ELEMS * 2
    steps_ms = hot_ms = float("nan")
    if args.main_only:  # profiling runs: nothing but the timed workload (+ warmup)
        plan.close()
        steps_plan.close()
        return {"ms_per_step": ms_per_step, "value": bytes_all / (ms_per_step * 1e-3) / 1e9}

    # schedule form (k_steps_reg: every RS / AG step of every rank in ONE persistent launch), same
    # buckets, timed like the headline's eager path: behind a spin kernel, R repetitions, median
    sched = timed_eager(stream, lambda: [step(i, steps_plan) for i in range(args.steps)], args.steps, reps)
    sched["launch"] = t.last_launch()
    steps_ms = sched["us_per_step"] * 1e-3

    # cache-resident (one bucket set, 40 MiB stays in the Infinity Cache)
    with torch.cuda.stream(stream):
        e0.record(stream)
        for i in range(args.steps):
            plan.execute(sets[0].data_ptr(), stride, None, stream)
        e1.record(stream)
    torch.cuda.synchronize()
    hot_ms = e0.elapsed_time(e1) / args.steps

    alg_bytes_hier = 2 * RANKS * ELEMS * 2
    # the N > 1 path's per-GPU step on this GPU alone (a one-rank peer set, W = 1): the
    # hierarchical step in one launch (k_hier_ws, the library default) and two buckets deep
    # (k_hier_x2: K buckets in K + 1 launches), same buckets, eager; no cross-GPU bytes at W = 1
    hier = {}
    try:
        peer = t.Peer(1, 0, 0, 2 * ELEMS)
        peer.connect([peer.handle()])
        ws_h = torch.empty(ELEMS, dtype=torch.int16, device=dev)
        # 8 rotating buckets of 64 contiguous rank rows (the peer calls' layout; 336 MB > the Infinity Cache)
        hsets = [torch.randint(0x3F80, 0x42C8, (RANKS, ELEMS), dtype=torch.int16, device=dev) for _ in range(8)]
        try:
            def one(i):
                peer.allreduce(hsets[i % 8].data_ptr(), ELEMS, stream, RANKS, SIDE, t.SWING, ws_h.data_ptr())

            def deep(k):
                for i in range(k):
                    peer.allreduce_pipelined2(hsets[i % 8].data_ptr(), ELEMS, stream)
                peer.allreduce_pipelined2(None, ELEMS, stream)

            for name, run_k in (("k_hier_ws", lambda k: [one(i) for i in range(k)]), ("k_hier_x2", deep)):
                with torch.cuda.stream(stream):   # warm: the headline's kernels ran last; >= 50 steps of this one
                    run_k(max(50, args.steps))
                torch.cuda.synchronize()
                # timed like the headline's eager path (behind a spin kernel that outlasts the host's
                # submission, R repetitions of K steps, the median; the pipelined form's finishing
                # launch inside every repetition); the grid the launcher chose and its residency beside it
                with torch.cuda.stream(stream):
                    r = timed_eager(stream, lambda: run_k(args.steps), args.steps, reps)
                    run_k(1)   # one more call: its launch is the one reported (a k_hier_x2 start, not a flush)
                r["launch"] = t.last_launch()
                torch.cuda.synchronize()
                r["hbm_frac"] = round(alg_bytes_hier / (r["us_per_step"] * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
                hier[name] = r
            hier["peer_status"] = peer.status()
        finally:
            peer.close()
            del hsets
    except Exception as e:  # reported, never silently dropped
        hier["error"] = repr(e)

    # host-staged end to end (buckets start and end in pinned host memory), the
    # reference program surface: H2D of all 64 buckets + allreduce + D2H, one DMA
    # each way ("dma"), or the fused kernel reading / writing the pinned host
    # buckets in place ("zerocopy")
    argv = ["allred_BO_2D", "1", "1", str(SIDE), "13", str(TILES), "32", "0", "1"]
    # ("dma": 8 column chunks, chunk c's H2D | pass | D2H overlapping the neighbours';
    # dma_chunks_<c> c chunks, 1 = one copy each way around one pass).  Each the median of 3 runs
    e2e = {}
    for mode, chunks in (("zerocopy", None), ("dma", None), ("dma_chunks_1", 1), ("dma_chunks_16", 16)):
        os.environ["ALLRED_E2E"] = "dma" if chunks or mode == "dma" else mode
        if chunks:
            os.environ["ALLRED_E2E_CHUNKS"] = str(chunks)
        try:
            e2e_runs = sorted((t.run(argv, t.BO, False, t.EXEC_FUSED) for _ in range(3)), key=lambda r: r.e2e_seconds)
            rep = e2e_runs[1]
            e2e[mode] = {"e2e_ms": round(rep.e2e_seconds * 1e3, 4), "device_ms": round(rep.device_seconds * 1e3, 4),
                         "value": round(bytes_all / rep.e2e_seconds / 1e9, 3),
                         "mismatches": int(max(r.mismatches for r in e2e_runs)),
                         "e2e_ms_runs": [round(r.e2e_seconds * 1e3, 4) for r in e2e_runs]}
        except Exception as e:  # reported, never silently dropped
            e2e[mode] = {"error": repr(e)}
        finally:
            del os.environ["ALLRED_E2E"]
            os.environ.pop("ALLRED_E2E_CHUNKS", None)

    # BASELINE config 1: 2x2 RecDub LO, 1 tile (2 kB per rank), seed -1 (all ones) —
    # latency-bound (no roofline): the fused one-launch plan, us per allreduce
    c1 = torch.full((4, 1024), 0x3F80, dtype=torch.int16, device=dev)   # bf16 1.0
    c1_plan = t.Plan(t.RECDUB, t.LO, 2, 1024, 4, t.EXEC_FUSED)
    with torch.cuda.stream(stream):
        for _ in range(20):
            c1.fill_(0x3F80)
            c1_plan.execute(c1.data_ptr(), 1024, None, stream)
    torch.cuda.synchronize()
    c1_ok = bool((c1 == 0x4080).all())   # every element = 4.0 (the known answer)
    c1_graph = None
    if not args.eager:   # the same launches replayed from a HIP graph (launch-bound: the graph is the faster)
        try:
            c1_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(c1_graph, stream=stream):
                for _ in range(args.steps):
                    c1_plan.execute(c1.data_ptr(), 1024, None, stream)
            torch.cuda.synchronize()
        except Exception as e:
            print(f"[bench] config-1 graph capture failed ({e}); eager", file=sys.stderr)
            c1_graph = None
    c1_us = {}
    for mode in ("eager", "graph"):
        if mode == "graph" and c1_graph is None:
            continue
        with torch.cuda.stream(stream):   # untimed pass first: the graph's first replay uploads it
            if mode == "graph":
                c1_graph.replay()
            else:
                for _ in range(args.steps):
                    c1_plan.execute(c1.data_ptr(), 1024, None, stream)
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            e0.record(stream)
            if mode == "graph":
                c1_graph.replay()
            else:
                for _ in range(args.steps):
                    c1_plan.execute(c1.data_ptr(), 1024, None, stream)
            e1.record(stream)
        torch.cuda.synchronize()
        c1_us[mode] = round(e0.elapsed_time(e1) / args.steps * 1e3, 3)
    c1_plan.close()
    config1 = {"workload": "2x2 RecDub LO, 1 tile (4 ranks x 2,048 B), seed -1; fused one-launch plan",
               "us_per_allreduce": c1_us.get("graph", c1_us["eager"]), "us_eager_launches": c1_us["eager"],
               "known_answer_ok": c1_ok, "note": "back-to-back allreduces on one stream: launch-bound, no roofline"}

    tsum = tilesum(stream, args.steps, reps)

    alg_bytes = 2 * RANKS * ELEMS * 2          # read every rank once, write every rank once
    achieved = alg_bytes / (ms_per_step * 1e-3) / 1e9
    out = {
        "metric": METRIC,
        "value": round(bytes_all / (ms_per_step * 1e-3) / 1e9, 3),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 6),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (uniform [0,100) bf16, reference rank convention); 32 rotating bucket sets in HBM (1.3 GB), "
                "rank rows 655,360 B + 128 B skew",
        "timing": {"method": "hip_graph_replays" if graph is not None else "eager_behind_spin_kernel",
                   "repetitions": reps, "ms_per_repetition": [round(x, 5) for x in rep_ms],
                   "ms_per_step": "median repetition / steps (each repetition = the K steps, back to back)"},
        "config": {"workload": "BASELINE config 2: 8x8 Swing BO allreduce, 64 virtual ranks x 655,360 B bf16 "
                               "(5 tiles/block) on one MI355X, fused one-pass HIP kernel, no RCCL",
                   "ranks": RANKS, "bytes_per_rank": ELEMS * 2, "algo": "swing", "variant": "BO",
                   "exec": "fused", "launches_per_step": plan.launches, "hip_graph": graph is not None},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": pmc_traffic(FUSED_KERNEL),
                     "kernel": FUSED_KERNEL, "algorithmic_bytes_per_launch": alg_bytes, "launch": fused_launch},
        "schedule_faithful": {"launches_per_step": steps_plan.launches, "ms_per_step": round(steps_ms, 6),
                              "value": round(bytes_all / (steps_ms * 1e-3) / 1e9, 3), **sched},
        "cache_resident": {"ms_per_step": round(hot_ms, 6), "value": round(bytes_all / (hot_ms * 1e-3) / 1e9, 3)},
        "hierarchical_step_w1": dict(hier, note="the N > 1 transports' per-GPU kernel on this GPU alone (one-rank peer "
                                     "set): tree of the 64 ranks, mem_2D hand-off, broadcast; eager launches behind a "
                                     "spin kernel, median of R repetitions of K steps"),
        "host_staged": e2e,
        "config1": config1,
        "tilesum": tsum,
        "prewarm_ms": round(prewarm_s * 1e3, 1),
        "host_wall_s": round(wall, 6),
    }
    plan.close()
    steps_plan.close()
    return out


def agreed_spin_cycles(stream, host_s: float) -> int:
    """torch.cuda._sleep cycles that outlast the slowest rank's host queueing of a timed
    region (host_s seconds on that rank): 3x the MAX over ranks + 200 us — the same spin on
    every rank, so no rank's timed region starts waiting for another's longer spin"""
    h = torch.tensor([host_s], dtype=torch.float64)
    dist.all_reduce(h, op=dist.ReduceOp.MAX)
    return int((3.0 * h.item() * 1e6 + 200.0) * spin_cycles_per_us(stream))


def timed_max(fn, reps, stream, after=None) -> float:
    """ms per call on `stream`, max over ranks.  after(): completes the calls
    (the pipelined transport's last bucket), inside the timed region.  The calls
    are queued behind a spin kernel sized from the warm calls' host time, so the
    GPU does not wait for the host inside the timed region (round 6; round 5's
    W = 1 k_hier_ws figure was such a wait)."""
    h0 = time.perf_counter()
    for _ in range(2):
        fn()
    if after:
        after()
    host_s = (time.perf_counter() - h0) / 2 * reps
    torch.cuda.synchronize()
    cycles = agreed_spin_cycles(stream, host_s)
    dist.barrier()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        torch.cuda._sleep(cycles)
    e0.record(stream)
    for _ in range(reps):
        fn()
    if after:
        after()
    e1.record(stream)
    torch.cuda.synchronize()
    m = torch.tensor([e0.elapsed_time(e1) / reps], dtype=torch.float64)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return m.item()


_SPIN_RATE = []


def spin_cycles_per_us(stream) -> float:
    """torch.cuda._sleep's cycles per microsecond on this GPU (measured once)"""
    if not _SPIN_RATE:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            torch.cuda._sleep(10000)
            e0.record(stream)
            torch.cuda._sleep(4000000)
            e1.record(stream)
        torch.cuda.synchronize()
        _SPIN_RATE.append(4000000 / max(1e-3, e0.elapsed_time(e1) * 1e3))
    return _SPIN_RATE[0]


def timed_eager(stream, run_rep, steps: int, reps: int) -> dict:
    """A secondary kernel timed like the headline's eager path: R repetitions of
    run_rep() (K steps, eager launches on `stream`) behind ONE spin kernel sized
    from a measured host submission rate so that it outlasts the host's queueing
    of every repetition, a HIP event between consecutive repetitions;
    us_per_step = the median repetition / K, with every repetition and the
    spread.  spin_covered_submission false = the host was still queueing when
    the GPU reached the timed region (then the numbers include host gaps)."""
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    with torch.cuda.stream(stream):
        run_rep()   # untimed: the host's cost of queueing one repetition
    host_s = time.perf_counter() - h0
    torch.cuda.synchronize()
    spin_us = 3.0 * host_s * 1e6 * reps + 500.0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    with torch.cuda.stream(stream):
        torch.cuda._sleep(int(spin_us * spin_cycles_per_us(stream)))
        ev[0].record(stream)
        h0 = time.perf_counter()
        for r in range(reps):
            run_rep()
            ev[r + 1].record(stream)
        submit_s = time.perf_counter() - h0
    torch.cuda.synchronize()
    per = [ev[r].elapsed_time(ev[r + 1]) * 1e3 / steps for r in range(reps)]
    return {"us_per_step": round(statistics.median(per), 3), "us_per_step_reps": [round(x, 3) for x in per],
            "spread_us": round(max(per) - min(per), 3), "repetitions": reps, "steps_per_repetition": steps,
            "host_submit_us_per_step": round(submit_s * 1e6 / (steps * reps), 3),
            "spin_us": round(spin_us, 1), "spin_covered_submission": submit_s * 1e6 < spin_us}


def prewarm(step, ms: float, batch: int = 50) -> float:
    """Untimed: run the workload for >= ms of wall time before the W warmup steps.
    A cold MI355X needs a few ms of sustained load to reach its steady clocks
    (config 2 measured 14.80-14.86 us per step after 20 warmup steps, 14.49-14.53
    after 1000); this makes the timed K steps measure the steady state whatever
    W the caller passes.  No timed step is skipped or shortened."""
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < ms * 1e-3:
        for _ in range(batch):
            step(i)
            i += 1
        torch.cuda.synchronize()
    return time.perf_counter() - t0


class Budget:
    """The N > 1 run's wall clock (--deadline, default 420 s: well under the
    driver's 600 s lease; counted from the start of bench.py, imports included).
    Records seconds per phase (xgmi.phase_s) and decides, agreed over ranks,
    when the remaining extras are skipped: a phase starts only while the budget
    left covers max(60 s, 2 x the longest phase so far).  The verified headline
    is measured first and is never skipped."""

    def __init__(self, deadline_s: float, t0: float):
        self.deadline, self.t0 = deadline_s, t0
        self.phase_s, self.skipped = {}, []
        self.longest = 0.0
        self.current = "start"   # the phase running now, or "after <phase>" (the watchdog's diagnosis)

    def elapsed(self) -> float:
        return time.perf_counter() - self.t0

    def left(self) -> float:
        return self.deadline - self.elapsed()

    @contextlib.contextmanager
    def phase(self, name: str):
        t0 = time.perf_counter()
        self.current = name
        if os.environ.get("ALLRED_BENCH_TEST_HANG_IN") == name:   # tests only: a host-side hang in this phase
            time.sleep(1e6)
        if os.environ.get("ALLRED_BENCH_TEST_RAISE_IN") == name:   # tests only: an error in this phase
            raise RuntimeError(f"test error in {name}")
        try:
            yield
        finally:
            d = time.perf_counter() - t0
            self.phase_s[name] = round(self.phase_s.get(name, 0.0) + d, 3)
            self.longest = max(self.longest, d)
            self.current = "after " + name

    def allows(self, name: str, agree: bool = True) -> bool:
        ok = self.left() > max(60.0, 2.0 * self.longest)
        if agree:   # every rank runs the same collectives: the most pressed rank decides
            ok = agreed(ok)
        if not ok:
            self.skipped.append(name)
        return ok

    def report(self) -> dict:
        return {"deadline_s": self.deadline, "wall_s": round(self.elapsed(), 3), "phase_s": dict(self.phase_s),
                "skipped_for_deadline": list(self.skipped), "phase_now": self.current,
                "rule": "a phase starts only while the budget left covers max(60 s, 2 x the longest phase so far)"}


def note(rank, msg):
    """progress line on stderr (stdout carries only the JSON line)"""
    print(f"[bench r{rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def agreed(ok: bool) -> bool:
    v = torch.tensor([int(ok)], dtype=torch.int64)
    dist.all_reduce(v, op=dist.ReduceOp.MIN)
    return bool(v.item())


# ---------------------------------------------------------------- N > 1 verification
# Every N > 1 transport is checked on the machine that times it, against values
# that do not come from any transport (validate_result_vector's role,
# allred_helper.cpp:18-120 / allred_helper.hpp:84-96):
#   exact_sum    every global row (GPU g, local rank l) gets 0 / 1 bf16 values drawn
#                from a hash of (seed, g * local + l, element) that every rank can
#                evaluate for every row, so each rank computes the exact sum of all
#                rows itself; counts stay <= 256, so every partial sum of every
#                reduction order is exact in bf16 and every correct transport
#                returns exactly that sum — a wrong, missing or doubled block shows.
#   closed_form  the reference's own inputs (even-x rows src_1, odd-x rows src_0,
#                allred_BO_2D.cpp:79-85), with the same a / b on every GPU.  On the
#                XOR schedules of the GPU grids every level of every rank's tree
#                combines two all-a / all-b / balanced groups, so the result is
#                exactly RNE(a + b) * R / 2 for R rows (the reference's expected
#                value, allred_helper.cpp:42-43, at error 0); mem_2D's fp32 sum
#                with one rounding gives the same bits.
MASK32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """32-bit integer finaliser on int64 tensors (constants < 2^31: no product
    leaves int64)"""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & MASK32
    x = x ^ (x >> 15)
    x = (x * 0x2C1B3C6D) & MASK32
    return x ^ (x >> 16)


def exact_bits_(out: torch.Tensor, row: int, seed: int, chunk: int = 1 << 24) -> None:
    """out (one row, int16 view of bf16) <- 1.0 with probability 1/4, else 0.0,
    a function of (seed, global row id, element index) only"""
    n = out.numel()
    key = _mix32(torch.tensor([(row * 0x9E3779B1 + seed * 0x632BE5AB + 1) & MASK32], dtype=torch.int64))
    key = key.to(out.device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        h = _mix32(torch.arange(s, e, dtype=torch.int64, device=out.device) ^ key)
        out[s:e] = torch.where((h & 3) == 0, 0x3F80, 0).to(torch.int16)


def exact_expected(rows: int, n: int, seed: int, dev) -> torch.Tensor:
    """int16 view of bf16: the exact sum over global rows 0 .. rows-1"""
    acc = torch.zeros(n, dtype=torch.int16, device=dev)
    tmp = torch.empty(n, dtype=torch.int16, device=dev)
    for r in range(rows):
        exact_bits_(tmp, r, seed)
        acc += (tmp != 0).to(torch.int16)
    if int(acc.max()) > 256:   # bf16 holds every integer up to 256 (never hit: mean rows / 4)
        raise RuntimeError("exact-sum inputs exceed 256 per element")
    return acc.to(torch.float32).to(torch.bfloat16).view(torch.int16)


def ref_pair(n: int, seed: int, dev):
    """src_0 / src_1 of the reference convention, identical on every rank (same seed)"""
    g = torch.Generator(device=dev).manual_seed(seed)
    a = (torch.rand(n, generator=g, device=dev) * 100).to(torch.bfloat16)
    b = (torch.rand(n, generator=g, device=dev) * 100).to(torch.bfloat16)
    return a, b


def closed_form(a: torch.Tensor, b: torch.Tensor, rows: int) -> torch.Tensor:
    """RNE(a + b) * rows / 2 (exact scaling by a power of two); one row: src_1 itself"""
    if rows == 1:
        return b.view(torch.int16)
    return ((a.float() + b.float()).to(torch.bfloat16) * (rows // 2)).view(torch.int16)


def verify_transport(run, buf: torch.Tensor, world: int, rank: int, local: int, local_side: int, side: int,
                     seed: int, status=None) -> dict:
    """run(buf) allreduces buf (local rows x n, in place) once; both checks, agreed
    over ranks (MIN): {"exact_sum": bool, "closed_form": bool, "verified": bool}.
    status(): nonzero when the transport itself reports a failure (peer timeout)."""
    n = buf.shape[1]
    rows = world * local
    res = {}
    err = None
    for check in ("exact_sum", "closed_form"):
        ok = True
        try:
            if check == "exact_sum":
                for l in range(local):
                    exact_bits_(buf[l], rank * local + l, seed)
                want = exact_expected(rows, n, seed, buf.device)
            else:
                a, b = ref_pair(n, seed + 1, buf.device)
                for l in range(local):   # x parity: the local grid's (hierarchical) or the GPU grid's (flat)
                    x = (l % local_side) if local > 1 else (rank % side)
                    buf[l].copy_((b if x % 2 == 0 else a).view(torch.int16))
                want = closed_form(a, b, rows)
                del a, b
            if buf.is_cuda:
                torch.cuda.synchronize(buf.device)
            run(buf)
            if buf.is_cuda:
                torch.cuda.synchronize(buf.device)
            ok = bool((buf == want[None, :]).all())
            if status is not None and status():
                ok = False
            del want
        except Exception as e:  # reported, never silently dropped: the check fails
            print(f"[bench r{rank}] verify {check}: {e!r}", file=sys.stderr)
            err = err or repr(e)
            ok = False
        res[check] = agreed(ok)
    res["verified"] = res["exact_sum"] and res["closed_form"]
    if err:   # e.g. a form the shape does not support (ALLRED_ERR_UNSUPPORTED): not a wrong result
        res["error"] = err[:200]
    return res


def open_peer(rank, world, local_rank, max_elems):
    """Peer windows (allred_peer_*), IPC handles exchanged over gloo.  Returns
    (peer, None) or (None, reason) — the same on every rank."""
    peer, mine = None, None
    try:
        peer = t.Peer(world, rank, local_rank, max_elems)
        mine = peer.handle()
    except Exception as e:  # every rank must learn of it, or the others block below
        print(f"[bench] peer create failed on rank {rank}: {e!r}", file=sys.stderr)
    handles = [None] * world
    dist.all_gather_object(handles, mine)
    if not all(h is not None for h in handles):
        if peer:
            peer.close()
        return None, "create failed on some rank"
    try:
        peer.connect(handles)
        ok = True
    except Exception as e:
        print(f"[bench] peer connect failed on rank {rank}: {e!r}", file=sys.stderr)
        ok = False
    if not agreed(ok):
        peer.close()
        return None, "connect failed on some rank"
    return peer, None


def bounded_frac(x, crossed: bool):
    """A roofline fraction as printed: null unless the bytes really crossed
    xGMI (not a --share-gpu rehearsal, where "remote" memory is local and the
    ratio means nothing) and 0 < x <= 1."""
    if not crossed or x is None or not (0 < x <= 1):
        return None
    return round(x, 4)


def arm_stats(ms, nbytes, world, lo=False, crossed=True) -> dict:
    """busbw = 2(p-1)/p * n / t (nccl-tests); xgmi_frac = busbw over this GPU's
    egress to its p-1 peers (one xGMI link each on the full mesh) at the spec
    per-direction link rate — bounded (bounded_frac)."""
    sec = ms * 1e-3
    busbw = 2 * (world - 1) / world * nbytes / sec / 1e9   # nccl-tests convention
    if lo:
        busbw = nbytes / sec / 1e9   # LO moves the whole bucket every step: report algbw
    return {"ms": round(ms, 4), "algbw_GBps": round(nbytes / sec / 1e9, 3), "busbw_GBps": round(busbw, 3),
            "xgmi_frac_spec": bounded_frac(busbw / (max(1, world - 1) * XGMI_LINK_DIR_GBPS), crossed)}


def roofline_xgmi(extras: dict, world: int, crossed: bool = True) -> dict | None:
    """The N > 1 xGMI roofline (north_star's >= 80 % target): the
    BASELINE config-4 arm (8-rank-grid Swing BO, 1 GiB of real bf16 per GPU, all
    links), the faster of its RCCL and peer-window transports among the arms
    VERIFIED on this machine, busbw over the GPU's egress = (p - 1) links x the
    MEASURED per-direction link rate (link_probe).  frac is null unless that
    peak was measured and 0 < frac <= 1 (a shared-GPU rehearsal has no link to
    measure: its numbers mean nothing); the spec-rate figure stays beside it."""
    arms = {k: v for k, v in extras.items() if "config4_swing_bo_1GiB_all_links" in k and isinstance(v, dict)
            and "busbw_GBps" in v and v.get("verified") is True and not v.get("peer_timeout")}
    if world < 2:
        return None
    if not arms:
        return {"bound": "xgmi", "achieved": None, "peak": None, "unit": "GB/s", "frac": None, "traffic": None,
                "note": "no verified config-4 arm"}
    name = max(arms, key=lambda k: arms[k]["busbw_GBps"])
    bus = arms[name]["busbw_GBps"]
    probe = extras.get("link_probe", {})
    link = probe.get("GBps_per_direction") if isinstance(probe, dict) else None
    peak_spec = (world - 1) * XGMI_LINK_DIR_GBPS
    peak = (world - 1) * link if link else None
    frac = bus / peak if peak else None
    sane = frac is not None and 0 < frac <= 1
    return {"bound": "xgmi", "achieved": bus, "peak": round(peak, 2) if peak else None, "unit": "GB/s",
            "frac": round(frac, 4) if sane else None, "traffic": None, "arm": name, "bytes_per_gpu": 1 << 30,
            "links": world - 1,
            "peak_source": "measured link_probe (RCCL sendrecv, both directions at once)" if link
                           else "not measured (no RCCL link probe: --share-gpu); frac null",
            "frac_unbounded": round(frac, 4) if frac is not None and not sane else None,
            "peak_spec": peak_spec, "frac_spec": bounded_frac(bus / peak_spec, crossed),
            "achieved_def": "busbw = 2(p-1)/p * bytes_per_gpu / t",
            # RCCL's own allreduce of the same 1 GiB per GPU (a comparator, not the product path)
            "rccl_allreduce_busbw": (extras.get("rccl_allreduce_comparator") or {}).get("config4_1GiB", {}).get(
                "busbw_GBps")}


def link_probe(rank, world, dev) -> dict:
    """Measured per-direction xGMI link rate (the xGMI-fraction
    denominator from an RCCL sendrecv microbench): ranks 2i <-> 2i+1 exchange
    128 MiB both ways at once over torch.distributed's nccl (= RCCL) backend."""
    pg = dist.new_group(backend="nccl")
    nbytes = 128 << 20
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    peer_rank = rank ^ 1

    def xchg():
        if peer_rank >= world:
            return
        ops = [dist.P2POp(dist.isend, a, peer_rank, group=pg), dist.P2POp(dist.irecv, b, peer_rank, group=pg)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()

    for _ in range(2):
        xchg()
    torch.cuda.synchronize()
    dist.barrier()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        xchg()
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    gbps = nbytes * reps / dt.item() / 1e9
    dist.destroy_process_group(pg)
    return {"bytes": nbytes, "reps": reps, "GBps_per_direction": round(gbps, 2),
            "spec_GBps_per_direction": XGMI_LINK_DIR_GBPS, "pairs": "2i<->2i+1, both directions at once"}


def rccl_allreduce_comparator(rank, world, dev, backend="nccl", sizes=None) -> dict:
    """RCCL's own ncclAllReduce (torch.distributed's nccl backend = RCCL), bf16 SUM, on config 3's
    640 kB and config 4's 1 GiB per GPU: an external comparator only, never the product path
    (SURVEY §8(e)).  Each size verified first (small integers 0..7 per element from a hash of
    (element, rank), so the sum is exact in any order), then timed like the arms (median of the
    reps' wall over ranks, MAX); busbw as nccl-tests.  (backend / sizes: the CPU test runs the
    same function over gloo on small buckets.)"""
    pg = dist.new_group(backend=backend)
    out = {}
    chunk = 1 << 26

    def sync():
        if torch.device(dev).type == "cuda":
            torch.cuda.synchronize()

    def ints_(x, r):   # x (bf16) <- the small integers of rank r
        for s0 in range(0, x.numel(), chunk):
            e = torch.arange(s0, min(x.numel(), s0 + chunk), dtype=torch.int64, device=dev)
            x[s0:s0 + e.numel()] = (((e * 2654435761 + r * 40503) >> 13) & 7).to(torch.bfloat16)

    try:
        for name, nbytes, reps in sizes or (("config3_640kB", ELEMS * 2, 50), ("config4_1GiB", 1 << 30, 5)):
            n = nbytes // 2
            x = torch.empty(n, dtype=torch.bfloat16, device=dev)
            want = torch.zeros(n, dtype=torch.bfloat16, device=dev)
            tmp = torch.empty_like(x)
            for r in range(world):
                ints_(tmp, r)
                want += tmp   # exact: every partial sum <= 56
            del tmp
            ints_(x, rank)
            dist.all_reduce(x, group=pg)
            sync()
            ok = agreed(bool(torch.equal(x, want)))
            del want
            for _ in range(2):
                dist.all_reduce(x, group=pg)
            sync()
            dist.barrier()
            per = []
            for _ in range(reps):
                t0 = time.perf_counter()
                dist.all_reduce(x, group=pg)
                sync()
                per.append(time.perf_counter() - t0)
            dt = torch.tensor([statistics.median(per)], dtype=torch.float64)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            out[name] = {**arm_stats(dt.item() * 1e3, nbytes, world), "verified_exact": ok, "reps": reps,
                         "op": "torch.distributed.all_reduce (RCCL ncclAllReduce), bf16 SUM"}
            del x
    finally:
        dist.destroy_process_group(pg)
    return out


def xgmi_arms(comm, peer, world, rank, dev, stream, side, total, crossed=True, budget=None) -> dict:
    """Flat / hierarchical inter-GPU allreduces (BASELINE configs 3-5 regimes),
    each through RCCL (allred_dist_allreduce) and through the peer windows
    (allred_peer_dist_allreduce: same program, same bits, one kernel), each
    verified on this machine before it is timed."""
    out = {}
    # BASELINE config 4: 8-rank Swing BO, 1 GiB per rank (all links = link-spreading channels; one link = plain)
    arms = [("config4_swing_bo_1GiB_all_links", t.SWING, t.BO, 1 << 30, 3, 0, 1),
            ("config4_swing_bo_1GiB_one_link", t.SWING, t.BO, 1 << 30, 2, 1, 1),
            ("swing_bo_256MiB_all_links", t.SWING, t.BO, 256 << 20, 5, 0, 1),
            ("config3_recdub_bo_640kB", t.RECDUB, t.BO, ELEMS * 2, 50, 0, 1),
            # the same bucket spread over every link (link-spreading channels; auto uses one below 1 MiB)
            ("config3_recdub_bo_640kB_all_links", t.RECDUB, t.BO, ELEMS * 2, 50, world - 1, 1),
            ("hierarchical_all_links", t.SWING, t.BO, ELEMS * 2, 50, world - 1, RANKS),
            ("hierarchical_lo_partial", t.SWING, t.LO, ELEMS * 2, 50, 1, RANKS)]
    # BASELINE config 5: flat 2D Swing LO, 2 kB .. 128 kB per GPU (latency regime)
    arms += [(f"config5_swing_lo_{kb}kB", t.SWING, t.LO, kb << 10, 100, 1, 1) for kb in (2, 8, 32, 128)]
    arms += [(f"mem_{kb}kB", t.SWING, t.MEM, kb << 10, 100, 1, 1) for kb in (2, 32)]
    arms += [("mem_640kB", t.SWING, t.MEM, ELEMS * 2, 100, 1, 1), ("mem_256MiB", t.SWING, t.MEM, 256 << 20, 5, 1, 1)]
    for arm in arms:
        if budget is not None and not budget.allows("arm:" + arm[0]):   # agreed over ranks
            continue
        # every arm runs the same calls with the same arguments on every rank, so an
        # error (an RCCL / HIP status turned exception) is raised on every rank alike:
        # record it, agree, and go on with the next arm instead of losing the line
        err = None
        try:
            with (budget.phase("arm:" + arm[0]) if budget is not None else contextlib.nullcontext()):
                xgmi_arm(out, comm, peer, world, rank, dev, stream, side, total, *arm, crossed=crossed)
        except Exception as e:  # reported, never silently dropped
            err = repr(e)
        if not agreed(err is None):
            out[arm[0] + "_error"] = err or "failed on another rank"
            torch.cuda.synchronize()
    out["best_per_config"] = best_arms(out)
    return out


def best_arms(out: dict) -> dict:
    """The fastest VERIFIED arm of each configuration over every transport and
    swept shape (RCCL, peer windows, grid sizes, LL / one-shot thresholds):
    what a tuned 8-GPU node would run for that bucket."""
    best = {}
    for key, v in out.items():
        if not isinstance(v, dict) or v.get("verified") is not True or "ms" not in v or v.get("peer_timeout"):
            continue
        cfg = key
        for pre in ("peer_sched_", "peer_oneshot_", "peer_push_", "peer_fenced_", "peer_"):
            if cfg.startswith(pre):
                cfg = cfg[len(pre):]
                break
        if cfg.startswith("g") and "_" in cfg and cfg.split("_", 1)[0][1:].isdigit():
            cfg = cfg.split("_", 1)[1]
        if cfg not in best or v["ms"] < best[cfg]["ms"]:
            best[cfg] = {"arm": key, "ms": v["ms"], "busbw_GBps": v.get("busbw_GBps")}
    return best


def xgmi_arm(out, comm, peer, world, rank, dev, stream, side, total, name, algo, variant, nbytes, reps, chans,
             local, crossed=True):
    """One arm of xgmi_arms: each transport verified (exact sums and the closed
    form, verify_transport), then timed on real data (uniform [0,100) bf16 per
    rank) into out[...] with its verdict beside the numbers."""
    n = nbytes // 2
    d2 = t.dist_desc(algo, variant, side, total, n, local_ranks=local, local_side=SIDE, local_algo=t.SWING,
                     channels=chans)
    b2 = torch.empty((local, n), dtype=torch.int16, device=dev)
    w2 = torch.empty(max(16, t.dist_workspace_bytes(d2)), dtype=torch.uint8, device=dev)
    seed = 5000 + 31 * len(out)

    def timed(key, fn, lo, status=None):
        v = verify_transport(fn, b2, world, rank, local, SIDE, side, seed, status=status)
        g = torch.Generator(device=dev).manual_seed(4000 + 17 * len(out) + rank)
        for r in range(local):   # real data for the timing
            b2[r].copy_((torch.rand(n, generator=g, device=dev) * 100).to(torch.bfloat16).view(torch.int16))
        ms = timed_max(lambda: fn(b2), reps, stream)
        out[key] = {**arm_stats(ms, nbytes, world, lo, crossed), "channels": chans, **v}

    if comm is not None and (variant != t.MEM or local == 1):   # mem_2D over RCCL: one rank per GPU
        timed(name, lambda b: t.dist_allreduce(comm, d2, b.data_ptr(), w2.data_ptr(), stream), variant == t.LO)
    if peer is not None:
        def status():
            return peer.status() & t.PEER_TIMEOUT

        def peer_fn(b):
            peer.dist_allreduce(d2, b.data_ptr(), w2.data_ptr(), stream)

        timed("peer_" + name, peer_fn, variant == t.LO, status)
        torch.cuda.synchronize()
        if status():   # sticky: this arm (or an earlier one) timed out, the numbers are void
            out["peer_" + name]["peer_timeout"] = True
            out["peer_" + name]["verified"] = False
        if variant != t.MEM and local == 1 and name.startswith(("config3", "config4")):
            # the scheduled form's grid is a guess (256 workgroups, 7 channels sharing
            # them): the same program at a quarter and a half of it, each a verified arm
            cap = 256 if crossed else 512 // world
            for groups in (cap // 4, cap // 2):
                peer.set_max_groups(groups)
                try:
                    timed(f"peer_g{groups}_" + name, peer_fn, variant == t.LO, status)
                    out[f"peer_g{groups}_" + name]["sched_groups"] = groups
                finally:
                    peer.set_max_groups(0 if crossed else cap)
            # the same program with every exchange pushed by the sender (k_peer_sched_push)
            peer.set_sched_push(1)
            try:
                timed("peer_push_" + name, peer_fn, variant == t.LO, status)
            finally:
                peer.set_sched_push(0)
            # the same program with tune peer_fence=1 (release / acquire fences around every flag)
            t.tune("peer_fence", 1)
            try:
                timed("peer_fenced_" + name, peer_fn, variant == t.LO, status)
            finally:
                t.tune("peer_fence", 0)
        if name.startswith("config5"):   # the same LO program without LL hand-offs (k_peer_sched)
            peer.set_lo_ll_max(0)
            try:
                timed("peer_sched_" + name, peer_fn, True, status)
            finally:
                peer.set_lo_ll_max(256 << 10)
        if variant == t.MEM and nbytes <= (256 << 10):   # mem_2D without LL hand-offs (k_peer_oneshot)
            peer.set_mem_ll_max(0)
            try:
                timed("peer_oneshot_" + name, peer_fn, False, status)
            finally:
                peer.set_mem_ll_max(256 << 10)
    del b2, w2


def cpu_baseline_multi() -> dict:
    """BASELINE configs 3, 4 and 5 in the oracle's loopback restatement (one forked
    process per rank, shared-memory buffers, semaphore handshakes) on this host's
    cores, 8 rank processes each (the 4x2 grid of the 8-GPU runs), as
    python/timing_taker.py runs each config beside its device run; ~15-25 s of CPU
    work in all.  value = config 3 (8 x 655,360 B over the median allreduce)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    cores = min(8, cpu_cores())

    def one(argv, budget_s, max_reps=400):
        probe = oracle.loopback("bo", argv, reps=2, total=8, timeout=300)
        reps = int(min(max_reps, max(3, budget_s / max(probe["median_s"], 1e-5))))
        out = oracle.loopback("bo", argv, reps=reps, total=8, timeout=300)
        nbytes = out["bytes_per_rank"]
        return {"us_median": round(out["median_s"] * 1e6, 3), "reps": reps, "bytes_per_rank": nbytes,
                "algbw_GBps": round(nbytes / out["median_s"] / 1e9, 4), "mismatches": out["mismatches"]}

    res = {}
    # config 3: allred_BO_2D 0 1 <4x2> 13 40 32 0 1 (RecDub BO, 40 tiles per block = 655,360 B per rank)
    res["config3_recdub_bo_640kB"] = c3 = one([0, 1, 4, 13, 40, 32, 0, 1], 4.0)
    # config 4 at a reduced bucket: 4096 tiles per block = 64 MiB per rank (1 GiB per rank
    # would hold 8 GiB of shared buffers; the CPU rate is flat in the bandwidth regime)
    res["config4_swing_bo_64MiB_reduced"] = one([1, 1, 4, 13, 4096, 32, 0, 1], 6.0, max_reps=5)
    for tiles, kb in ((1, 2), (4, 8), (16, 32), (64, 128)):   # config 5: Swing LO 2 .. 128 kB
        res[f"config5_swing_lo_{kb}kB"] = one([1, 1, 4, 13, tiles, 32, 0, 0], 2.0)
    return {"value": round(8 * c3["bytes_per_rank"] / (c3["us_median"] * 1e-6) / 1e9, 4), "unit": "GB/s",
            "cores": cores, "kind": "port",
            "sample": ("oracle loopback, 8 forked rank processes per config (4x2 grid): config 3 RecDub BO "
                       "640 kB, config 4 Swing BO at 64 MiB per rank (reduced from 1 GiB, <= 5 reps), "
                       "config 5 Swing LO 2/8/32/128 kB; value = config 3, bytes of all 8 ranks / median time"),
            "online_cpus": os.sysconf("SC_NPROCESSORS_ONLN"), "configs": res}


def dropped_candidates(verify: dict) -> list:
    """xgmi.dropped: every transport whose verdict is not verified, with why —
    a peer wait that gave up in its quick timing, bits that differ from the
    form of the same semantics, a failed exact-sum / closed-form check."""
    out = []
    for kind, v in verify.items():
        if v.get("verified") is True:
            continue
        if v.get("quick_timing_timeout"):
            why = "quick_timing_timeout: a peer wait gave up during its timing"
        elif any(k.startswith("matches_") and v[k] is False for k in v):
            why = "differs from " + next(k[len("matches_"):] for k in v if k.startswith("matches_") and v[k] is False)
        elif v.get("exact_sum") is False:
            why = "exact_sum check failed"
        elif v.get("closed_form") is False:
            why = "closed_form check failed"
        else:
            why = "verification failed"
        out.append({"transport": kind, "reason": why})
    return out


def choose_transport(quick: dict, verify: dict):
    """The fastest transport whose verdict is verified (None if none is)."""
    ok = [k for k in quick if verify.get(k, {}).get("verified") is True]
    return min(ok, key=lambda k: quick[k]) if ok else None


def cli_config3(world: int, share: bool = False) -> dict:
    """BASELINE config 3 through the reference's own program surface on every GPU
    of this node: bin/allred_BO_2D 0 1 4 13 40 32 0 1 with ALLRED_NODES=8 (the 4x2
    grid) and ALLRED_GPUS = the GPUs this process sees (one device thread per GPU,
    RCCL between them), every GPU's ranks checked with validate_result_vector.
    share (--share-gpu rehearsal): ALLRED_GPUS = world groups on the one GPU over
    the in-process peer windows (ALLRED_TRANSPORT=peer, ALLRED_SHARE_GPU=1), the
    same G-thread orchestration with the exchange the hardware allows."""
    gpus = world if share else min(world, torch.cuda.device_count())
    env = {"ALLRED_NODES": "8", "ALLRED_GPUS": str(gpus), "ALLRED_REPORT": "1", "ALLRED_CHECK_ALL": "1",
           "ALLRED_STRICT": "1"}
    if share:
        env.update({"ALLRED_TRANSPORT": "peer", "ALLRED_SHARE_GPU": "1", "GPU_MAX_HW_QUEUES": "16"})
    argv = [0, 1, 4, 13, 40, 32, 0, 1]
    p = t.run_cli("allred_BO_2D", argv, env=env, timeout=180)
    rep = {}
    for line in p.stderr.splitlines():
        if line.startswith("{"):
            rep = json.loads(line)
    ok = p.returncode == 0 and "All values match!" in p.stdout and rep.get("mismatches") == 0
    out = {"argv": " ".join(map(str, ["allred_BO_2D", *argv])), "env": env, "rc": p.returncode, "verified": ok,
           "report": rep}
    if rep.get("device_s"):
        out["algbw_GBps"] = round(rep["bytes_per_rank"] / rep["device_s"] / 1e9, 3)
        out["busbw_GBps"] = round(2 * 7 / 8 * rep["bytes_per_rank"] / rep["device_s"] / 1e9, 3)
    if not ok:
        out["stderr_tail"] = p.stderr[-400:]
    return out


def bench_multi(args, rank, world, local_rank, emit) -> dict | None:
    budget = Budget(args.deadline, _T0)
    BUDGET[0] = budget
    setup = budget.phase("setup")
    setup.__enter__()
    # --share-gpu (rehearsal only): every rank on cuda:0 and no RCCL (it refuses two
    # ranks on one device), so the whole N>1 path except RCCL runs on a 1-GPU box
    dev_index = 0 if args.share_gpu else local_rank
    dev = torch.device(f"cuda:{dev_index}")
    torch.cuda.set_device(dev)
    side, total = GRIDS[world]
    comm, comm_err = None, None
    if not args.share_gpu:
        try:   # RCCL communicator (allred_dist_comm_create); without it the peer transports still run
            uid = [t.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = t.Comm(uid[0], world, rank, local_rank)
        except Exception as e:  # reported in the line (xgmi.rccl_error), never silently dropped
            comm_err = repr(e)
            note(rank, f"RCCL communicator failed: {comm_err}")
        if not agreed(comm is not None):
            if comm is not None:
                comm.close()
            comm, comm_err = None, comm_err or "failed on another rank"
    stream = torch.cuda.Stream(device=dev)
    desc = t.dist_desc(t.SWING, t.BO, side, total, ELEMS, local_ranks=RANKS, local_side=SIDE, local_algo=t.SWING)
    # rotating bucket sets as at N = 1 (every step streams its 64 ranks from HBM)
    bufs = [torch.empty((RANKS, ELEMS), dtype=torch.int16, device=dev) for _ in range(args.sets)]
    for i, b in enumerate(bufs):
        fill_reference_convention(b, 77 + rank + 1000 * i)
    buf = bufs[0]
    torch.cuda.synchronize()
    ws = torch.empty(t.dist_workspace_bytes(desc), dtype=torch.uint8, device=dev)
    partial = torch.empty(ELEMS, dtype=torch.int16, device=dev)
    partial2 = torch.zeros(ELEMS, dtype=torch.int16, device=dev)
    ws2 = torch.empty(2 * t.dist_workspace_bytes(desc), dtype=torch.uint8, device=dev)   # rccl_x: two parities
    vbuf = torch.empty((RANKS, ELEMS), dtype=torch.int16, device=dev)   # verification bucket
    t_start = time.perf_counter()
    setup.__exit__(None, None, None)

    def timed_steps(step_fn, after=None, reps=None):
        """R repetitions of the K steps behind a spin kernel, an event between
        consecutive ones; per repetition the max over ranks; returns (median ms
        per step, every repetition's ms per step)"""
        reps = reps or max(3, min(args.reps, 5))
        torch.cuda.synchronize()
        dist.barrier()
        # one untimed repetition: the host's cost of queueing K steps sizes the spin kernel
        # below (the same on every rank), so the GPU never waits for the host in the timed region
        h0 = time.perf_counter()
        for i in range(args.steps):
            step_fn(i)
        if after is not None:
            after()
        host_s = (time.perf_counter() - h0) * reps
        torch.cuda.synchronize()
        cycles = agreed_spin_cycles(stream, host_s)
        dist.barrier()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        with torch.cuda.stream(stream):
            torch.cuda._sleep(cycles)
        ev[0].record(stream)
        for r in range(reps):
            for i in range(args.steps):
                step_fn(i)
            if after is not None:
                after()
            ev[r + 1].record(stream)
        torch.cuda.synchronize()
        dist.barrier()
        ms = torch.tensor([ev[r].elapsed_time(ev[r + 1]) for r in range(reps)], dtype=torch.float64)
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        per = [m / args.steps for m in ms.tolist()]
        return statistics.median(per), per

    def local_phases_ms(fused=False):
        """the HBM kernels of the launch transports alone, ms per step: the tree
        reduce of the 64 ranks + the broadcast of the same bucket (rccl,
        peer_swing), or (fused) bucket i+1's tree and bucket i's broadcast in one
        pass (k_tree_bcast_x, rccl_x)"""
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(args.steps):
            b = bufs[i % len(bufs)]
            if fused:
                nb = bufs[(i + 1) % len(bufs)]
                t.tree_broadcast_pipelined(nb.data_ptr(), b.data_ptr(), ELEMS, ELEMS, t.SWING, SIDE, RANKS,
                                           partial.data_ptr(), partial2.data_ptr(), stream)
            else:   # the partial alternates between two buffers, as in allred_dist_allreduce
                pp = (partial, partial2)[i & 1]
                t.tree_reduce(b.data_ptr(), ELEMS, ELEMS, t.SWING, SIDE, RANKS, pp.data_ptr(), stream)
                t.broadcast(b.data_ptr(), ELEMS, ELEMS, RANKS, pp.data_ptr(), stream)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.steps

    # Inter-GPU transport: the candidates for the hierarchical step
    #   rccl        tree -> 2D Swing BO over RCCL -> broadcast (3 launches + RCCL groups)
    #   rccl_x      the same, consecutive buckets pipelined: bucket i's broadcast and bucket
    #               i+1's tree in ONE pass (k_tree_bcast_x), then bucket i+1's RCCL program
    #   peer_launches  tree -> mem_2D across GPUs over peer windows (launches) -> broadcast: verified,
    #               the bit-identity reference of the one-kernel forms, not a candidate
    #   peer_swing  tree -> the same Swing program over peer windows (k_peer_sched) -> broadcast
    #   peer_mem_x  consecutive buckets pipelined: bucket i's broadcast and bucket i+1's tree in
    #               one pass (k_tree_bcast_x), then bucket i+1's partial through the one-kernel
    #               mem_2D exchange over the peer windows (k_peer_oneshot)
    #   peer_hier_ws  ONE kernel: tree -> mem_2D across GPUs -> broadcast, every cross-GPU
    #                 hand-off an LL push; reducing and writing waves in every workgroup
    #                 (k_hier_ws: 14.5-14.7 us at W = 1)
    #   peer_hier_x2t2  two buckets deep (k_hier_x2: launch i reads bucket i, sums bucket i-1's
    #                 owned tiles before its last row stores, writes bucket i-2; every poll waits
    #                 for the previous launch)
    #   peer_swing_fenced / peer_mem_x_fenced  the same kernels with tune peer_fence=1: a
    #                 system-scope release fence before every flag store, an acquire fence after
    #                 every flag wait (same bits; the form that stays correct on a node that breaks
    #                 the ordering argument of DESIGN.md §5).  The LL forms have no separate flag
    # (retired, every measurement slower — profiles/README.md: in round 5 the per-tile flag
    # form k_hier_oneshot, the pipelined LL form k_hier_pipe, the flag hand-off forms; in
    # round 6 k_hier_ll (16.2 us at W = 1), the one-deep pipeline k_hier_x (15.1-15.3) and
    # k_hier_x2's other placements)
    # Every transport runs only once verified on THIS machine (verify_transport: the
    # exact sum of per-row 0/1 inputs and the reference's closed form, both computed
    # without any transport); the one-kernel peer forms must also equal the launch
    # form of the same semantics bit for bit on random real data, and peer_swing the
    # RCCL program's.  Then each verified one is timed and the fastest is the headline.
    peer_box = [None]
    mode = [None]   # the peer form currently set (set only on change: the timed loop is one C call a step)
    pend2 = [False]   # peer_hier_x2t2: the kind whose buckets are started and not finished (flush())
    pend3 = [False]   # rccl_x: a bucket is started and not finished (flush())
    pend4 = [None, 0]   # peer_mem_x: the started bucket and the partial slot it used (flush())
    mem_parts = [torch.empty(ELEMS, dtype=torch.int16, device=dev) for _ in range(2)]
    fence = [None]
    ws_mem = torch.empty(ELEMS, dtype=torch.int16, device=dev)

    def set_fence(v):   # tune peer_fence, read at every peer launch
        if fence[0] != v:
            t.tune("peer_fence", v)
            fence[0] = v

    def flush():
        peer = peer_box[0]
        if pend3[0]:
            t.dist_allreduce_pipelined(comm, desc, None, ws2.data_ptr(), stream)
            pend3[0] = False
        if pend4[0] is not None:
            t.broadcast(pend4[0], ELEMS, ELEMS, RANKS, mem_parts[pend4[1]].data_ptr(), stream)
            pend4[0] = None
        if pend2[0]:
            peer.allreduce_pipelined2(None, ELEMS, stream)
            pend2[0] = False

    def run(kind, b, fresh=False):
        peer = peer_box[0]
        if fresh:   # b was just written on torch's current stream
            stream.wait_stream(torch.cuda.current_stream())
        if kind.startswith("peer"):   # <kind>_fenced: the same kernel with the fences
            base = kind[:-len("_fenced")] if kind.endswith("_fenced") else kind
            set_fence(int(base != kind))
            kind = base
        if kind == "rccl_x":   # buckets pipelined: this call writes the previous one's rows
            if pend2[0] or pend4[0] is not None:
                flush()
            t.dist_allreduce_pipelined(comm, desc, b.data_ptr(), ws2.data_ptr(), stream)
            pend3[0] = True
            return
        if kind == "peer_mem_x":   # buckets pipelined: this call writes the previous one's rows
            if pend2[0] or pend3[0]:
                flush()
            if mode[0] != kind:
                peer.set_oneshot_max(4 << 20)
                peer.set_hier_ll(0)
                mode[0] = kind
            slot = pend4[1] ^ 1 if pend4[0] is not None else 0
            out = mem_parts[slot]
            if pend4[0] is None:
                t.tree_reduce(b.data_ptr(), ELEMS, ELEMS, t.SWING, SIDE, RANKS, out.data_ptr(), stream)
            else:
                t.tree_broadcast_pipelined(b.data_ptr(), pend4[0], ELEMS, ELEMS, t.SWING, SIDE, RANKS, out.data_ptr(),
                                           mem_parts[pend4[1]].data_ptr(), stream)
            peer.allreduce(out.data_ptr(), ELEMS, stream)   # the partial: mem_2D across the GPUs
            pend4[0], pend4[1] = b.data_ptr(), slot
            return
        if kind in X2_KINDS:   # two deep: this call writes the bucket started two calls ago
            if pend3[0] or pend4[0] is not None or (pend2[0] and pend2[0] != kind):
                flush()
            peer.allreduce_pipelined2(b.data_ptr(), ELEMS, stream)
            pend2[0] = kind
            return
        flush()
        if kind == "rccl":
            t.dist_allreduce(comm, desc, b.data_ptr(), ws.data_ptr(), stream)
        elif kind == "peer_swing":
            peer.dist_allreduce(desc, b.data_ptr(), ws.data_ptr(), stream)
        else:
            if mode[0] != kind:
                peer.set_oneshot_max(0 if kind == "peer_launches" else (4 << 20))
                peer.set_hier_ll(1 if kind == "peer_hier_ws" else 0)
                mode[0] = kind
            peer.allreduce(b.data_ptr(), ELEMS, stream, RANKS, SIDE, t.SWING, ws_mem.data_ptr())

    verify = {}
    comparator = {}   # peer_launches: verified like a candidate, the bit-identity reference of the one-kernel forms

    def check(kind, seed):
        with budget.phase("verify:" + kind):
            return check_(kind, seed)

    def check_(kind, seed):
        note(rank, f"verify: {kind}")
        peer = peer_box[0]

        def once(b):
            run(kind, b, fresh=True)
            flush()

        status = (lambda: peer.status() & t.PEER_TIMEOUT) if kind.startswith("peer") else None
        v = verify_transport(once, vbuf, world, rank, RANKS, SIDE, side, seed, status=status)
        base = kind[:-len("_fenced")] if kind.endswith("_fenced") else kind
        same_as = {"peer_swing": "rccl", "rccl_x": "rccl"}.get(base, None if base in ("rccl", "peer_launches")
                                                                     else "peer_launches")
        if same_as == "rccl" and not verify.get("rccl", {}).get("verified"):
            same_as = None   # --share-gpu: no RCCL to compare with (the Swing trees differ from mem_2D's)
        if same_as == "peer_launches" and not comparator.get("peer_launches", {}).get("verified"):
            same_as = None   # the comparator itself did not verify (its own checks stand)
        if v["verified"] and same_as:   # random real data: bit-identical to the form of the same semantics
            ok = False
            try:
                a, b2 = buf.clone(), buf.clone()
                run(same_as, a, fresh=True)
                run(kind, b2)
                flush()
                torch.cuda.synchronize()
                ok = torch.equal(a, b2) and not (status and status())
                del a, b2
            except Exception as e:  # reported, never silently dropped: the candidate is not used
                note(rank, f"verify: {kind} vs {same_as} raised {e!r}")
            v["matches_" + same_as] = agreed(ok)
            v["verified"] = v["matches_" + same_as]
        verify[kind] = v
        note(rank, f"verify: {kind} -> {v}")
        return v["verified"]

    # RCCL first, verified before any number of it is measured: the watchdog's
    # fallback line below is only ever an RCCL number that passed both checks
    rccl_ok = comm is not None and check("rccl", 9000)
    rccl_x_ok = rccl_ok and check("rccl_x", 9050)
    peer_guard = None
    if rccl_ok:
        note(rank, "fallback headline over RCCL")
        for i in range(args.warmup):
            run("rccl", bufs[i % len(bufs)])
        fb_ms, _ = timed_steps(lambda i: run("rccl", bufs[i % len(bufs)]))
        fb_local = local_phases_ms()
        FALLBACK_DONE.set()
        BEST_LINE[0] = lambda: multi_line(args, world, "rccl", fb_ms, fb_local, time.perf_counter() - t_start,
                                          {"headline_transport": "rccl", "transport_verified": dict(verify),
                                           "budget": budget.report()})

        # the peer phase may take --peer-timeout s, and never past the deadline (less the extras' margin)
        peer_limit = max(30.0, min(args.peer_timeout, budget.left() - 90.0))

        def peer_give_up():
            if rank == 0:
                emit(multi_line(args, world, "rccl", fb_ms, fb_local, time.perf_counter() - t_start,
                                {"headline_transport": "rccl", "transport_verified": dict(verify), "peer_error":
                                 f"peer setup / verification / timing did not finish within {peer_limit:g} s",
                                 "budget": budget.report()}))
            os._exit(0)

        # every rank's timer started after the same barrier: all leave together; a rank
        # whose own timer was cancelled first and then loses rank 0 exits cleanly too
        # (FALLBACK_DONE, main())
        peer_guard = threading.Timer(peer_limit, peer_give_up)
        peer_guard.daemon = True
        peer_guard.start()
    note(rank, f"world {world}, device {dev_index}: opening peer windows")
    peer, peer_err = open_peer(rank, world, dev_index, (1 << 30) // 2)   # windows for 1 GiB buckets
    peer_box[0] = peer
    note(rank, f"peer windows: {'ok' if peer is not None else peer_err}")
    if peer is not None and args.share_gpu:
        peer.set_max_groups(512 // world)   # every rank's one-kernel grid resident at once
    if peer is None and not rccl_ok:
        raise RuntimeError("no verified transport: RCCL " + (comm_err or ("unverified" if comm else "absent")) +
                           f", peer windows: {peer_err}")
    def drop(kind, reason):   # on stderr as it happens; xgmi.dropped lists them all (dropped_candidates)
        note(rank, f"DROPPED {kind}: {reason}")

    candidates = (["rccl"] if rccl_ok else []) + (["rccl_x"] if rccl_x_ok else [])
    for kind, ok in (("rccl", rccl_ok), ("rccl_x", rccl_x_ok)):
        if comm is not None and kind in verify and not ok:
            drop(kind, "verification failed")
    quick = {}
    # each candidate timed the way the headline is: K steps with the pipelined forms'
    # finishing launch inside (it weighs 1/K per step), median of three
    qk = max(args.steps, 10)

    def quick_time(kinds):
        for kind in kinds:
            with budget.phase("quick:" + kind):
                quick_time1(kind)

    def quick_time1(kind):
        note(rank, f"quick timing: {kind}")
        it = iter(range(1 << 30))
        quick[kind] = round(statistics.median(
            timed_max(lambda: run(kind, bufs[next(it) % len(bufs)]), qk, stream, after=flush)
            for _ in range(3)), 4)
        if peer is not None and kind.startswith("peer"):
            # a peer wait that gave up means wrong bytes: the candidate is out (every rank agrees),
            # and the sticky status bit is cleared so the next candidates wait normally again
            torch.cuda.synchronize()
            st0 = torch.tensor([peer.status() & t.PEER_TIMEOUT], dtype=torch.int64)
            dist.all_reduce(st0, op=dist.ReduceOp.MAX)
            if st0.item():
                drop(kind, "quick_timing_timeout: a peer wait gave up during its timing")
                quick.pop(kind, None)
                verify.setdefault(kind, {}).update(verified=False, quick_timing_timeout=True)
                peer.clear_status()
                dist.barrier()

    quick_time(list(candidates))
    if peer is not None:
        # the launch form (tree, mem_2D exchange as launches, broadcast) first: not a candidate
        # (slower than every one-kernel form in every measurement), the form the one-kernel
        # forms must equal bit for bit on random data
        check("peer_launches", 9090)
        comparator["peer_launches"] = verify.pop("peer_launches")
        relaxed = ("peer_swing", "peer_mem_x", "peer_hier_ws", *X2_KINDS)
        passed = []
        for i, kind in enumerate(relaxed):
            if check(kind, 9100 + 10 * i):
                passed.append(kind)
            else:
                drop(kind, "verification failed")
        quick_time(passed)
        # the fenced twins of the flag-protocol forms, so a node that breaks the relaxed
        # ordering still leaves a verified peer form behind
        fenced = []
        for i, kind in enumerate(FLAG_KINDS):
            if check(kind + "_fenced", 9300 + 10 * i):
                fenced.append(kind + "_fenced")
            else:
                drop(kind + "_fenced", "verification failed")
        quick_time(fenced)
        set_fence(0)
    if not quick:
        raise RuntimeError(f"no transport passed verification on this machine: {verify}")
    transport = choose_transport(quick, verify)
    if transport is None:   # every verified candidate had a peer wait give up in its timing
        raise RuntimeError(f"no transport timed without a peer timeout on this machine: {verify}")

    def step(i):
        run(transport, bufs[i % len(bufs)])

    note(rank, f"timed: {transport}")
    headline_phase = budget.phase("headline")
    headline_phase.__enter__()
    # untimed prewarm (steady clocks): the SAME number of steps on every rank — the
    # ranks' calls must pair up (RCCL collectives, peer epochs) — derived from the
    # max-over-ranks quick timing, identical everywhere
    pre_steps = int(min(20000, args.prewarm_ms / max(quick[transport], 1e-3)))
    for i in range(pre_steps):
        step(i)
    for i in range(args.warmup):
        step(i)
    flush()
    t0 = time.perf_counter()
    # rccl_x / peer_mem_x / peer_hier_x2t2: the finishing launch is part of each repetition's K steps
    ms_per_step, rep_ms = timed_steps(step, after=flush)
    wall = time.perf_counter() - t0
    peer_timeout = False
    if transport != "rccl" and peer is not None:
        # a timed-out peer wait means wrong bytes: such a number is never the headline
        st0 = torch.tensor([peer.status() & t.PEER_TIMEOUT], dtype=torch.int64)
        dist.all_reduce(st0, op=dist.ReduceOp.MAX)
        peer_timeout = bool(st0.item())
        if peer_timeout:
            if not rccl_ok:
                raise RuntimeError(f"peer transport {transport} timed out during the timed steps: no valid number")
            note(rank, f"{transport} timed out in the timed loop: timing the RCCL transport instead")
            transport = "rccl_x" if rccl_x_ok and quick.get("rccl_x", 1e9) < quick.get("rccl", 1e9) else "rccl"
            for i in range(args.warmup):
                step(i)
            ms_per_step, rep_ms = timed_steps(step, after=flush)
    if peer is not None:   # defaults again for the extras below
        peer.set_oneshot_max(4 << 20)
        peer.set_hier_ll(0)
        set_fence(0)
        mode[0] = None
    headline_phase.__exit__(None, None, None)
    fused_local = transport in ("rccl_x", "peer_mem_x")
    with budget.phase("local_phases"):
        local_ms = local_phases_ms(fused=fused_local)
        local_split_ms = local_phases_ms() if fused_local else local_ms
    if peer_guard is not None:   # the headline is measured: the extras have their own watchdog
        peer_guard.cancel()
    HEADLINE_DONE.set()

    extras = {"headline_transport": transport, "transport_verified": verify, "transport_quick_ms": quick,
              "dropped": dropped_candidates(verify), "comparator_verified": comparator,
              "peer_timeout_in_timed_loop": peer_timeout,
              "local_phases_ms": {"tree_then_broadcast": round(local_split_ms, 6),
                                  **({"tree_broadcast_fused": round(local_ms, 6)} if fused_local else {})},
              "timing": {"repetitions": len(rep_ms), "ms_per_step_per_repetition": [round(x, 6) for x in rep_ms],
                         "ms_per_step": "median repetition (each: the K steps, max over ranks)"}}
    if peer_err:
        extras["peer_error"] = peer_err
    if comm_err:
        extras["rccl_error"] = comm_err

    def line(ex):
        return multi_line(args, world, transport, ms_per_step, local_ms, wall, ex)

    def best_line():   # the headline with the extras gathered so far (main()'s last-resort watchdog)
        try:
            ex = {k: v for k, v in list(extras.items())}
        except Exception:  # extras being written concurrently: headline only
            ex = {}
        ex["budget"] = budget.report()
        return line(ex)

    BEST_LINE[0] = best_line

    if args.extras:
        # The headline is measured; the extras must not be able to lose it.  If
        # they have not finished after --extras-timeout s (a hung transport on an
        # untried machine), rank 0 prints the line with what it has and every
        # rank leaves; the driver still gets its one JSON line.
        def give_up():
            if rank == 0:
                try:
                    ex = {k: v for k, v in list(extras.items())}
                except Exception:  # extras being written concurrently: headline only
                    ex = {}
                ex["extras_error"] = f"extras did not finish within {extras_limit:g} s"
                ex["budget"] = budget.report()
                emit(line(ex))
            os._exit(0)

        # the extras end by the deadline whatever happens (rank 0 prints the line with what it has)
        extras_limit = max(10.0, min(args.extras_timeout, budget.left() - 15.0))
        guard = threading.Timer(extras_limit + (0 if rank == 0 else 10), give_up)
        guard.daemon = True
        guard.start()
        extras.update(xgmi_arms(comm, peer if verify.get("peer_swing", {}).get("verified") else None, world, rank,
                                dev, stream, side, total, crossed=not args.share_gpu, budget=budget))
        if world > 1 and comm is not None and budget.allows("link_probe"):
            try:
                with budget.phase("link_probe"):
                    extras["link_probe"] = link_probe(rank, world, dev)
                mb = extras["link_probe"]["GBps_per_direction"]
                for v in extras.values():  # the fraction again against the MEASURED link rate
                    if isinstance(v, dict) and "busbw_GBps" in v:
                        v["xgmi_frac_measured_link"] = bounded_frac(v["busbw_GBps"] / ((world - 1) * mb),
                                                                    not args.share_gpu)
            except Exception as e:  # reported, never silently dropped
                extras["link_probe"] = {"error": repr(e)}
        if world > 1 and comm is not None and budget.allows("rccl_allreduce_comparator"):
            try:
                with budget.phase("rccl_allreduce_comparator"):
                    extras["rccl_allreduce_comparator"] = rccl_allreduce_comparator(rank, world, dev)
                mb = extras.get("link_probe", {}).get("GBps_per_direction")
                if mb:
                    for v in extras["rccl_allreduce_comparator"].values():
                        v["xgmi_frac_measured_link"] = bounded_frac(v["busbw_GBps"] / ((world - 1) * mb), True)
            except Exception as e:  # reported, never silently dropped
                extras["rccl_allreduce_comparator"] = {"error": repr(e)}
        guard.cancel()
    if peer is not None:
        st = torch.tensor([peer.status()], dtype=torch.int64)
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        extras["peer_status"] = int(st.item())
        dist.barrier()
        peer.close()
    if comm is not None:
        comm.close()
    del bufs, vbuf, ws, ws2
    torch.cuda.synchronize()
    # rank 0 alone (the others wait at the barrier): the reference's program surface
    # across this node's GPUs (config 3), then the CPU baseline of configs 3-5
    # (rank 0 alone: the others wait at the barrier, so no agreement is needed)
    if rank == 0 and args.extras and budget.allows("cli_config3", agree=False):
        try:
            with budget.phase("cli_config3"):
                extras["cli_config3"] = cli_config3(world, share=args.share_gpu)
        except Exception as e:  # reported, never silently dropped
            extras["cli_config3"] = {"error": repr(e), "verified": False}
    cpu = None
    if rank == 0 and args.cpu and budget.allows("cpu_baseline", agree=False):
        try:
            with budget.phase("cpu_baseline"):
                cpu = cpu_baseline_multi()
        except Exception as e:  # reported, never silently dropped
            cpu = {"value": None, "error": repr(e)}
    dist.barrier()
    if rank != 0:
        return None
    extras["budget"] = budget.report()
    out = line(extras)
    if cpu is not None:
        out["cpu_baseline"] = cpu
    return out


# the N > 1 run's budget and the best line it could print so far (a callable: the RCCL fallback
# once measured, then the headline with the extras gathered so far), for main()'s last-resort watchdog
BUDGET = [None]
BEST_LINE = [None]
# rank 0's one JSON line goes out once, whichever of the normal path and the watchdogs gets there first
EMITTED = threading.Event()
_EMIT_LOCK = threading.Lock()


def watchdog_line(args, world: int, reason: str) -> dict:
    """What rank 0 prints when the N > 1 run cannot finish its line (reason): main()'s
    last-resort watchdog (a host-side hang no phase watchdog covers: RCCL setup or
    verification before the fallback is measured, teardown) or an exception: the best line
    measured so far with xgmi.watchdog, else a line with value null and the phase it was in."""
    b = BUDGET[0]
    where = b.current if b is not None else "before the N > 1 setup"
    msg = f"{reason} (phase: {where})"
    ln = None
    if BEST_LINE[0] is not None:
        try:
            ln = BEST_LINE[0]()
        except Exception as e:  # reported below, never silently dropped
            msg += f"; the measured line could not be rebuilt: {e!r}"
    if ln is not None:
        ln.setdefault("xgmi", {})["watchdog"] = msg
        return ln
    return {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"config 2 per GPU (64 virtual ranks x 655,360 B, 8x8 Swing) x {world} GPUs",
                       "parallelism": f"dp{world}"},
            "error": msg, "xgmi": {"budget": b.report() if b is not None else None}}


# set once the N > 1 headline is measured: a rank that then loses its peers
# (rank 0 gave up on the extras and left) exits cleanly instead of failing the job
HEADLINE_DONE = threading.Event()
# set once the RCCL fallback line is measured: rank 0's peer watchdog may then print
# it and leave while this rank's own (already cancelled) timer did not fire
FALLBACK_DONE = threading.Event()

# the one-launch kernel of each one-kernel transport (its HBM bytes over the step time)
ONE_LAUNCH = {"peer_hier_ws": "k_hier_ws", "peer_hier_x2t2": "k_hier_x2"}
# the k_hier_x2 transports (owned sums before a launch's last row stores)
X2_KINDS = ("peer_hier_x2t2",)
# the transports whose cross-GPU hand-offs are data + a separate flag (k_peer_sched, k_peer_oneshot):
# their tune peer_fence=1 twins are candidates too
FLAG_KINDS = ("peer_swing", "peer_mem_x")


def multi_line(args, world, transport, ms_per_step, local_ms, wall, extras) -> dict:
    """rank 0's JSON line of the N > 1 bench"""
    bytes_all = world * RANKS * ELEMS * 2
    local_bytes = 2 * RANKS * ELEMS * 2 + 2 * ELEMS * 2
    fenced = transport.endswith("_fenced")   # the same kernel with tune peer_fence=1
    base = transport[:-len("_fenced")] if fenced else transport
    if base in ONE_LAUNCH:   # the step IS one launch: its HBM bytes over its time
        kern = ONE_LAUNCH[base]
        roof = {"kernel": f"{kern} (whole step)", "algorithmic_bytes_per_launch": 2 * RANKS * ELEMS * 2,
                "achieved": 2 * RANKS * ELEMS * 2 / (ms_per_step * 1e-3) / 1e9, "traffic": pmc_traffic(kern)}
    elif base in ("rccl_x", "peer_mem_x"):   # the local HBM pass: bucket i's broadcast + i+1's tree, one kernel
        roof = {"kernel": "k_tree_bcast_x (local phases of consecutive buckets, one pass)",
                "algorithmic_bytes_per_launch": local_bytes, "achieved": local_bytes / (local_ms * 1e-3) / 1e9,
                "traffic": pmc_traffic("k_tree_bcast_x<1>")}
    else:
        tr, bc = pmc_traffic("k_tree_lds_pipe<64, false>"), pmc_traffic("k_broadcast")
        roof = {"kernel": "k_tree_lds_pipe<64, false> + k_broadcast (local phases)",
                "algorithmic_bytes_per_launch": local_bytes, "achieved": local_bytes / (local_ms * 1e-3) / 1e9,
                "traffic": tr + bc if tr and bc else None}
    achieved = roof["achieved"]
    via = {"rccl": "on-GPU tree reduce, 2D Swing BO over RCCL/xGMI, broadcast",
           "peer_mem_x": "consecutive buckets pipelined (K buckets in K + 1 calls, all inside the timed region): "
                         "bucket i's broadcast and bucket i+1's on-GPU tree reduce in one HBM pass, then bucket i+1's "
                         "partial through the one-kernel mem_2D exchange over peer-mapped xGMI windows",
           "rccl_x": "consecutive buckets pipelined (K buckets in K + 1 calls, all inside the timed region): "
                     "bucket i's broadcast and bucket i+1's on-GPU tree reduce in one HBM pass, then bucket i+1's "
                     "2D Swing BO over RCCL/xGMI",
           "peer_launches": "on-GPU tree reduce, mem_2D across GPUs over peer-mapped windows (launches), broadcast",
           "peer_swing": "on-GPU tree reduce, 2D Swing BO over peer-mapped xGMI windows (one kernel), broadcast",
           "peer_hier_x2t2": "ONE kernel per bucket, two buckets deep (K buckets in K + 1 launches, all inside the "
                             "timed region): launch i reads bucket i, writes bucket i-2's rows and, before its last "
                             "row stores, sums bucket i-1's owned tiles; mem_2D one-shot across GPUs with LL pushes "
                             "into peer-mapped xGMI windows",
           "peer_hier_ws": "ONE kernel: on-GPU tree reduce, mem_2D one-shot across GPUs with LL pushes "
                           "(data+epoch words) into peer-mapped xGMI windows, broadcast; every workgroup's reducing "
                           "waves stream tiles in while its writing waves write finished tiles' rows"}[base]
    if fenced:
        via += " (peer_fence: release / acquire fences around every cross-GPU hand-off)"
    v = extras.get("transport_verified", {}).get(transport, {})
    return {
        "metric": METRIC,
        "value": round(bytes_all / (ms_per_step * 1e-3) / 1e9, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 6),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": f"synthetic (uniform [0,100) bf16, reference rank convention); {args.sets} rotating bucket sets per GPU",
        "config": {"workload": f"config 2 per GPU (64 virtual ranks x 655,360 B, 8x8 Swing) x {world} GPUs: "
                               f"{via}; GPU grid {GRIDS[world]}",
                   "ranks": RANKS * world, "bytes_per_rank": ELEMS * 2, "parallelism": f"dp{world}",
                   "transport": transport, "verified": v.get("verified") is True},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": roof["traffic"], "kernel": roof["kernel"],
                     "algorithmic_bytes_per_launch": roof["algorithmic_bytes_per_launch"],
                     # the PMC pass runs on one GPU: at W > 1 the hand-off words add to it
                     "traffic_source": "profiles/pmc_traffic.json, measured at W = 1",
                     "local_phases_ms": round(local_ms, 6)},
        "roofline_xgmi": roofline_xgmi(extras, world, crossed=not args.share_gpu),
        "xgmi": extras,
        "host_wall_s": round(wall, 6),
    }


def main():
    # RCCL and gloo print banners on stdout; keep stdout for the one JSON line
    real_stdout = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--prewarm-ms", type=float, default=50.0,
                    help="untimed sustained load before the warmup steps (steady clocks); 0 = none")
    ap.add_argument("--sets", type=int, default=32, help="rotating bucket sets (1.3 GB per GPU: far past the 256 MiB MALL)")
    ap.add_argument("--eager", action="store_true", help="no HIP graph capture")
    ap.add_argument("--reps", type=int, default=5,
                    help="N = 1: back-to-back replays of the K timed steps; ms_per_step = median replay / K")
    ap.add_argument("--no-cpu-baseline", dest="cpu", action="store_false")
    ap.add_argument("--no-extras", dest="extras", action="store_false")
    ap.add_argument("--peer-timeout", type=float, default=240.0,
                    help="N > 1: seconds the peer-window phase may take before the RCCL-measured line is printed")
    ap.add_argument("--extras-timeout", type=float, default=240.0,
                    help="N > 1: seconds the extras may take before the headline line is printed without them")
    ap.add_argument("--deadline", type=float, default=420.0,
                    help="N > 1: seconds from the start of bench.py by which the line is printed; the extras "
                         "after the verified headline are skipped as the deadline nears (xgmi.budget)")
    ap.add_argument("--main-only", action="store_true", help="timed workload only (for rocprofv3 runs)")
    ap.add_argument("--tilesum-only", type=int, nargs="*", default=None, metavar="MIB",
                    help="only the tile-sum part of the N = 1 line, at these sizes in MiB (default 256 1024; "
                         "for rocprofv3 runs)")
    ap.add_argument("--force-dist", action="store_true", help="run the N>1 code path on one GPU (1-rank RCCL)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal: every rank on cuda:0, peer transports only (no RCCL); not a measurement")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.force_dist:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            dist.init_process_group("gloo", rank=0, world_size=1)
        else:
            dist.init_process_group("gloo")
        def emit(line):   # rank 0's one line, whoever gets there first
            with _EMIT_LOCK:
                if EMITTED.is_set():
                    return
                sys.stdout.flush()
                os.write(real_stdout, (json.dumps(line) + "\n").encode())
                EMITTED.set()

        # last resort: the phase watchdogs (peer phase, extras) cover the hangs they can fall back
        # from; anything else (RCCL setup / verification before the fallback, teardown) ends here,
        # --deadline + 120 s after bench.py started (the driver's lease is 600 s), with a line
        hard_s = float(os.environ.get("ALLRED_BENCH_HARD_S", args.deadline + 120.0))

        def last_resort():
            code = 0
            if rank == 0 and not EMITTED.is_set():
                ln = watchdog_line(args, world, f"the N > 1 run had not printed its line {hard_s:.0f} s after "
                                                "bench.py started")
                note(rank, ln.get("error") or ln["xgmi"]["watchdog"])
                emit(ln)
                code = 0 if ln.get("value") is not None else 1
            sys.stderr.flush()
            os._exit(code)

        # rank 0 first: the others leave 15 s later, so rank 0's line is not lost to their exit
        hard = threading.Timer(max(1.0, hard_s - (time.perf_counter() - _T0)) + (0 if rank == 0 else 15),
                               last_resort)
        hard.daemon = True
        hard.start()
        try:
            out = bench_multi(args, rank, world, local_rank, emit)
        except Exception as e:
            if rank == 0:   # still one line: the best measured so far, else value null and the error
                traceback.print_exc()
                ln = watchdog_line(args, world, f"the N > 1 run raised {e!r}")
                emit(ln)
                sys.stderr.flush()
                os._exit(0 if ln.get("value") is not None else 1)
            if not (HEADLINE_DONE.is_set() or FALLBACK_DONE.is_set()):
                raise
            note(rank, f"ended by a peer's exit ({e!r}); rank 0 reports the line")
            sys.stderr.flush()
            os._exit(0)
        if out is not None:
            emit(out)
            out = None
        dist.destroy_process_group()
    elif args.tilesum_only is not None:
        sizes = [m << 20 for m in (args.tilesum_only or [256, 1024])]
        out = {"tilesum": tilesum(torch.cuda.Stream(device="cuda:0"), args.steps, max(1, args.reps), sizes)}
    else:
        out = bench_single(args)
        if args.cpu and not args.main_only:
            try:
                out["cpu_baseline"] = cpu_baseline()
            except Exception as e:  # reported, never silently dropped
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if out is not None:
        sys.stdout.flush()
        os.write(real_stdout, (json.dumps(out) + "\n").encode())


if __name__ == "__main__":
    main()
