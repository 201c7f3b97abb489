#!/usr/bin/env python3
"""Copy-speed reference for the fused pass: device-to-device copies of the
config-2 footprint (64 x 655,360 B = 41.9 MB read + 41.9 MB written), 8
rotating buffer pairs, HIP-graph replay — the floor a one-pass allreduce
that reads and writes every byte once can approach.  Also k_add (tile-sum)
and k_copy_ranks at the same size.  One JSON line per arm."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

nbytes = 64 * 655360
n = nbytes // 2
src = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(8)]
dst = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(8)]
s = torch.cuda.Stream()


def timed(fn, steps=200):
    with torch.cuda.stream(s):
        for i in range(10):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(steps):
            fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    with torch.cuda.stream(s):
        g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e3


us = timed(lambda i: dst[i % 8].copy_(src[i % 8]))
print(json.dumps({"arm": "torch_copy_42MB", "us": round(us, 3), "GBps": round(2 * nbytes / us / 1e3, 1)}))
us = timed(lambda i: t.bf16_add(dst[i % 8].data_ptr(), src[i % 8].data_ptr(), n, s))
print(json.dumps({"arm": "k_add_42MB", "us": round(us, 3), "GBps": round(3 * nbytes / us / 1e3, 1)}))
