#!/usr/bin/env python3
"""k_hier_x at W = 1: per bucket, the pipelined sequence (one launch reads
bucket i+1 and writes bucket i) vs the same work unpipelined (a read-only
launch then a write-only launch per bucket) — does the overlap happen?
python tools/hier_x_probe.py [buckets]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
P, n, NS = 64, 327680, 32
sets = [torch.randint(0x3F80, 0x42C8, (P, n), dtype=torch.int16, device="cuda") for _ in range(NS)]
peer = t.Peer(1, 0, 0, 2 * n)
peer.connect([peer.handle()])
s = torch.cuda.Stream()


def pipelined():
    prev = None
    for i in range(K):
        cur = sets[i % NS].data_ptr()
        peer.allreduce_pipelined(cur, prev, n, s)
        prev = cur
    peer.allreduce_pipelined(None, prev, n, s)


def split():
    for i in range(K):
        cur = sets[i % NS].data_ptr()
        peer.allreduce_pipelined(cur, None, n, s)
        peer.allreduce_pipelined(None, cur, n, s)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(3):
        with torch.cuda.stream(s):
            torch.cuda._sleep(20000000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        out.append(round(e0.elapsed_time(e1) * 1e3 / K, 3))
    return out


res = {"pipelined_us_per_bucket": timed(pipelined), "split_us_per_bucket": timed(split)}
peer.close()
print(json.dumps(res))
