#!/usr/bin/env python3
"""Host-link probe for the end-to-end (buckets in pinned host memory) path:
DMA H2D / D2H alone and together, kernel reads / writes of pinned host
memory, and the fused BO pass on host buckets (zero-copy) — one JSON line
per arm.  Usage: python tools/pcie_probe.py [grid_cap]  (ALLRED_PIPE_GRID)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

N_BYTES = 64 * 655360
n = N_BYTES // 2
dev = torch.device("cuda:0")
s = torch.cuda.Stream()
s2 = torch.cuda.Stream()
h = torch.zeros(n, dtype=torch.int16).pin_memory()
h2 = torch.zeros(n, dtype=torch.int16).pin_memory()
d = torch.zeros(n, dtype=torch.int16, device=dev)
d2 = torch.zeros(n, dtype=torch.int16, device=dev)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def emit(name, ms, nbytes):
    print(json.dumps({"arm": name, "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 2)}), flush=True)


with torch.cuda.stream(s):
    emit("dma_h2d", timed(lambda: d.copy_(h, non_blocking=True)), N_BYTES)
    emit("dma_d2h", timed(lambda: h.copy_(d, non_blocking=True)), N_BYTES)


def both():
    ev = torch.cuda.Event()
    ev.record(s)
    s2.wait_event(ev)
    d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)
    ev2 = torch.cuda.Event()
    ev2.record(s2)
    s.wait_event(ev2)


with torch.cuda.stream(s):
    emit("dma_both_directions", timed(both), 2 * N_BYTES)
    # kernel reads host: d += h (host read n*2; HBM traffic ignored)
    emit("kernel_read_host", timed(lambda: t.bf16_add(d.data_ptr(), h.data_ptr(), n, s)), N_BYTES)
    # kernel writes host: broadcast one device row to one host row
    emit("kernel_write_host", timed(lambda: t.broadcast(h.data_ptr(), n, n, 1, d.data_ptr(), s)), N_BYTES)
    # kernel read+write host: h += d2 (reads h, writes h)
    emit("kernel_rw_host", timed(lambda: t.bf16_add(h.data_ptr(), d2.data_ptr(), n, s)), 2 * N_BYTES)
    hb = torch.zeros((64, 327680), dtype=torch.int16).pin_memory()
    plan = t.Plan(t.SWING, t.BO, 8, 327680, 64, t.EXEC_FUSED)
    emit(f"fused_bo_zero_copy_grid{os.environ.get('ALLRED_PIPE_GRID', '512')}",
         timed(lambda: plan.execute(hb.data_ptr(), 327680, None, s), 10), 2 * N_BYTES)
    plan.close()
