#!/usr/bin/env python3
"""Timing of the hierarchical local phases (64 virtual ranks x 640 kB per GPU):
tree reduce to one partial, broadcast back, both, and bucket i's broadcast
fused with bucket i+1's tree (k_tree_bcast_x, the rccl_x transport) — rotating bucket sets,
HIP graph replay, the bench.py method.  Env knobs (ALLRED_TREE=lds, ...) pass
through for A/B.   python tools/hier_local.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
P, n = 64, 327680
NS = int(os.environ.get("AB_SETS", "32"))
sets = [torch.randint(0x3F80, 0x42C8, (P, n), dtype=torch.int16, device="cuda") for _ in range(NS)]
outs = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(NS)]
s = torch.cuda.Stream()


def tree(i):
    t.tree_reduce(sets[i % NS].data_ptr(), n, n, t.SWING, 8, P, outs[i % NS].data_ptr(), s)


def bcast(i):
    t.broadcast(sets[i % NS].data_ptr(), n, n, P, outs[i % NS].data_ptr(), s)


def both(i):
    tree(i)
    bcast(i)


def fused(i):   # bucket i's broadcast (from its result) + bucket i+1's tree, one pass
    t.tree_broadcast_pipelined(sets[(i + 1) % NS].data_ptr(), sets[i % NS].data_ptr(), n, n, t.SWING, 8, P,
                               outs[(i + 1) % NS].data_ptr(), outs[i % NS].data_ptr(), s)


res = {}
for name, fn, nbytes in (("tree", tree, P * n * 2 + n * 2), ("broadcast", bcast, P * n * 2 + n * 2),
                         ("tree+broadcast", both, 2 * (P * n * 2 + n * 2)),
                         ("tree_bcast_x", fused, 2 * (P * n * 2 + n * 2))):
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
    us = e0.elapsed_time(e1) / steps * 1e3
    res[name] = {"us": round(us, 3), "hbm_GBps": round(nbytes / us / 1e3, 1)}
print(json.dumps({"local_phases": res, "env": {k: v for k, v in os.environ.items() if k.startswith(("ALLRED_", "AB_"))}}))
