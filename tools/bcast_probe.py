#!/usr/bin/env python3
"""Why k_broadcast runs longer inside the peer launch form (W = 1 hier step,
rocprofv3: 13.7 us) than alone (7.8 us): the same 64 x 640 kB buckets (32
rotating sets) through (A) broadcast alone, (B) tree -> broadcast, (C) tree ->
peer mem_2D launches (copy, barrier, reduce-scatter, barrier, all-gather) ->
broadcast, (D) tree -> a tiny peer call -> broadcast, (E) as B with the
broadcast's source another buffer, (F) as B writing a bucket the tree did not
just read, (G) B's launches replayed from a HIP graph, (H) as B with a partial
buffer per bucket set (tools/hier_local.py's pattern), (I) / (J) as B with the
partial alternating over 2 / 4 buffers.  Prints event-timed us
per step of the eager arms.  Run under rocprofv3
--kernel-trace: per-kernel durations by arm (arms run in order, K steps each).
   python tools/bcast_probe.py [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
P, n, NS = 64, 327680, 32
sets = [torch.randint(0x3F80, 0x42C8, (P, n), dtype=torch.int16, device="cuda") for _ in range(NS)]
ws = torch.empty(n, dtype=torch.int16, device="cuda")
NO_PEER = os.environ.get("NO_PEER") == "1"   # no peer windows in the process: arms C and D skipped
peer = None
if not NO_PEER:
    peer = t.Peer(1, 0, 0, 2 * n)
    peer.connect([peer.handle()])
    peer.set_oneshot_max(0)   # the multi-launch mem_2D form
s = torch.cuda.Stream()
ws2 = torch.empty(n, dtype=torch.int16, device="cuda")
outs = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(NS)]   # H: a partial per set (hier_local)
ev = {}
# E: the broadcast's source is NOT the partial the tree just wrote; F: the broadcast writes
# a bucket set the tree did NOT just read; G: B's launches captured in a HIP graph
for arm in ("A", "B", "E", "F", "G", "H", "I", "J") if NO_PEER else ("A", "B", "C", "D", "E", "F", "G", "H", "I", "J"):
    def one(i):
        b = sets[i % NS]
        part = {"H": outs[i % NS], "I": outs[i % 2], "J": outs[i % 4]}.get(arm, ws)
        if arm in "BCDEFGHIJ":
            t.tree_reduce(b.data_ptr(), n, n, t.SWING, 8, P, part.data_ptr(), s)
        if arm == "C":
            peer.allreduce(ws.data_ptr(), n, s)   # the partial through the peer launches (W = 1)
        if arm == "D":
            peer.allreduce(ws[:64].data_ptr(), 64, s)   # a tiny peer call: its barriers, no bytes
        dst = sets[(i + NS // 2) % NS] if arm == "F" else b
        t.broadcast(dst.data_ptr(), n, n, P, (ws2 if arm == "E" else part).data_ptr(), s)
    if arm == "G":
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(steps):
                one(i)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            g.replay()
    else:
        for i in range(10):
            one(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            torch.cuda._sleep(5000000)
        e0.record(s)
        for i in range(steps):
            one(i)
        e1.record(s)
        torch.cuda.synchronize()
        ev[arm] = round(e0.elapsed_time(e1) * 1e3 / steps, 2)
    torch.cuda.synchronize()
print("us_per_step_events", ev)
if peer is not None:
    print("peer_status", peer.status())
    peer.close()
