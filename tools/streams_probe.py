#!/usr/bin/env python3
"""Do consecutive config-2 allreduces of INDEPENDENT buckets gain from running
on two streams (the tail of bucket i's persistent grid overlapping the head of
bucket i+1's)?  Same plan, 32 rotating bucket sets, eager launches behind a
spin kernel, K steps: one stream (the bench) vs two alternating streams joined
at the end (an event on the second stream waited for by the first).
   python tools/streams_probe.py [steps] [rounds]"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
P, n, NS = 64, 327680, 32
stride = t.preferred_rank_stride(n)
sets = [torch.randint(0x3F80, 0x42C8, (P, stride), dtype=torch.int16, device="cuda") for _ in range(NS)]
plan = t.Plan(t.SWING, t.BO, 8, n, P, t.EXEC_FUSED)
s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
res = {"one_stream": [], "two_streams": []}
for _ in range(rounds):
    for arm in res:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s0):
            torch.cuda._sleep(5000000)
        e0.record(s0)
        s1.wait_event(e0)
        for i in range(steps):
            st = s1 if (arm == "two_streams" and i % 2) else s0
            plan.execute(sets[i % NS].data_ptr(), stride, None, st)
        if arm == "two_streams":
            j = torch.cuda.Event()
            j.record(s1)
            s0.wait_event(j)
        e1.record(s0)
        torch.cuda.synchronize()
        res[arm].append(round(e0.elapsed_time(e1) * 1e3 / steps, 3))
print(json.dumps({"us_per_allreduce": res, "median": {k: statistics.median(v) for k, v in res.items()},
                  "steps": steps, "sets": NS}))
plan.close()
