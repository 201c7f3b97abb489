#!/usr/bin/env python3
"""Timing of the hierarchical step on ONE GPU (W = 1 peer set, 64 virtual ranks
x 640 kB): the launch form (tree + mem_2D + broadcast), k_hier_ws (and its A/B
column splits / load depth) and k_hier_x2 (buckets pipelined two deep: K buckets
in K + 1 launches, the timed region includes the finishing launch) — the N > 1
bench's candidates with the cross-GPU hand-offs reduced to this GPU's own boxes.  Eager launches behind a spin
kernel (peer calls advance host-side epochs, so no graph), 32 rotating sets,
arms interleaved.   python tools/hier_step.py [steps] [rounds]   (HIER_CAP: grid cap)"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
P, n = 64, 327680
NS = int(os.environ.get("AB_SETS", "32"))
sets = [torch.randint(0x3F80, 0x42C8, (P, n), dtype=torch.int16, device="cuda") for _ in range(NS)]
ws = torch.empty(n, dtype=torch.int16, device="cuda")
peer = t.Peer(1, 0, 0, 2 * n)
peer.connect([peer.handle()])
peer.set_max_groups(int(os.environ.get("HIER_CAP", "0")))   # 0: the default grid (2 workgroups per CU)
s = torch.cuda.Stream()
arms = {"launches": (0, 0), "oneshot_exchange": (1 << 40, 0), "hier_ws": (0, 1),
        "hier_ws_a2": (0, 1), "hier_ws_c8": (0, 1), "hier_ws_c8_a2": (0, 1),
        "hier_ws_c32": (0, 1), "hier_ws_c32_a2": (0, 1)}
# hier_ws_a2: tune hier_ws_ahead=2; _c8 / _c32: hier_ws_cols=8 / 32 (quarter / whole tiles per reducing wave;
# default 16: halves)
# the pipelined arm: k_hier_x2, two buckets deep
PIPE = ["hier_x2"]
if os.environ.get("HIER_ARMS"):   # a subset, comma separated (any of the names above)
    sel = os.environ["HIER_ARMS"].split(",")
    arms = {k: v for k, v in arms.items() if k in sel}
    PIPE = [k for k in sel if k.startswith("hier_x2")]
res = {k: [] for k in list(arms) + PIPE}
host = {k: [] for k in res}   # host submission time per call: must stay below the GPU time
SPIN = int(os.environ.get("SPIN_CYCLES", "20000000"))   # the GPU busy until the host has queued every step
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def pipelined(k):   # k buckets in k + 1 calls (k_hier_x2)
    for i in range(k):
        peer.allreduce_pipelined2(sets[i % NS].data_ptr(), n, s)
    peer.allreduce_pipelined2(None, n, s)


for _ in range(rounds):
    for name in PIPE:
        pipelined(20)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            torch.cuda._sleep(SPIN)
        e0.record(s)
        h0 = time.perf_counter()
        pipelined(steps)
        host[name].append(round((time.perf_counter() - h0) * 1e6 / steps, 2))
        e1.record(s)
        torch.cuda.synchronize()
        res[name].append(round(e0.elapsed_time(e1) * 1e3 / steps, 3))
    for name, (limit, ll) in arms.items():
        peer.set_oneshot_max(limit)
        peer.set_hier_ll(ll)
        t.tune("hier_ws_ahead", 2 if name.endswith("_a2") else 1)
        t.tune("hier_ws_cols", 8 if "_c8" in name else 32 if "_c32" in name else 16)
        for i in range(20):
            peer.allreduce(sets[i % NS].data_ptr(), n, s, P, 8, t.SWING, ws.data_ptr())
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            torch.cuda._sleep(SPIN)
        e0.record(s)
        h0 = time.perf_counter()
        for i in range(steps):
            peer.allreduce(sets[i % NS].data_ptr(), n, s, P, 8, t.SWING, ws.data_ptr())
        host[name].append(round((time.perf_counter() - h0) * 1e6 / steps, 2))
        e1.record(s)
        torch.cuda.synchronize()
        res[name].append(round(e0.elapsed_time(e1) * 1e3 / steps, 3))
status = peer.status()
peer.close()
print(json.dumps({"W": 1, "bytes_per_rank": n * 2, "ranks": P, "sets": NS, "steps": steps,
                  "us_per_step": res, "median": {k: statistics.median(v) for k, v in res.items()},
                  "host_us_per_call": host, "spin_cycles": SPIN,
                  "peer_status": status}))
