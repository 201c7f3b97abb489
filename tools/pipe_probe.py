#!/usr/bin/env python3
"""Probe: the hierarchical step's two HBM phases of CONSECUTIVE bucket sets on
two streams (bucket i's broadcast beside bucket i+1's tree reduce), one GPU,
64 virtual ranks x 640 kB, 32 rotating sets.  The exchange of the partial
(N > 1) would sit between them; here it is absent (W = 1).  Reports us per
step for: tree + broadcast on one stream, the two-stream pipeline, and the
fused one-pass kernel for reference.   python tools/pipe_probe.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
P, n = 64, 327680
NS = 32
R = 3   # partial ring
sets = [torch.randint(0x3F80, 0x42C8, (P, n), dtype=torch.int16, device="cuda") for _ in range(NS)]
parts = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(R)]
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
plan = t.Plan(t.SWING, t.BO, 8, n, P, t.EXEC_FUSED)


def tree(i, st):
    t.tree_reduce(sets[i % NS].data_ptr(), n, n, t.SWING, 8, P, parts[i % R].data_ptr(), st)


def bcast(i, st):
    t.broadcast(sets[i % NS].data_ptr(), n, n, P, parts[i % R].data_ptr(), st)


def one_stream():
    for i in range(K):
        tree(i, s1)
        bcast(i, s1)


def fused():
    for i in range(K):
        plan.execute(sets[i % NS].data_ptr(), n, None, s1)


def two_streams():
    done = [None] * K
    ready = [None] * K
    for i in range(K):
        if i >= R:   # the partial slot is free once bucket i-R was broadcast
            s1.wait_event(done[i - R])
        tree(i, s1)
        ready[i] = torch.cuda.Event()
        ready[i].record(s1)
        s2.wait_event(ready[i])
        bcast(i, s2)
        done[i] = torch.cuda.Event()
        done[i].record(s2)
    s1.wait_stream(s2)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(3):
        with torch.cuda.stream(s1):
            torch.cuda._sleep(400000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s1)
        s2.wait_stream(s1)
        fn()
        s1.wait_stream(s2)
        e1.record(s1)
        torch.cuda.synchronize()
        best.append(round(e0.elapsed_time(e1) * 1e3 / K, 3))
    return best


out = {"steps": K, "one_stream_us": timed(one_stream), "two_streams_us": timed(two_streams), "fused_us": timed(fused)}
# correctness of the pipelined form: the last bucket equals its one-stream result
ref = sets[(K - 1) % NS].clone()
print(json.dumps(out))
plan.close()
