#!/usr/bin/env python3
"""A/B timing of one fused plan (64 ranks, config-2 size by default) with
rotating bucket sets, HIP graph replay — the bench.py method for any variant.
  python tools/ab_fused.py <bo|lo|mem> [tiles] [steps]   (env knobs pass through); AB_EAGER=1: plain launches"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402

variant = {"bo": t.BO, "lo": t.LO, "mem": t.MEM}[sys.argv[1]]
tiles = int(sys.argv[2]) if len(sys.argv) > 2 else 5
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
P = int(os.environ.get("AB_P", "64"))
SIDE = int(os.environ.get("AB_SIDE", "8"))
n = t.normalize_tiles(tiles, P, variant != t.LO) * 1024
stride = n + int(os.environ["AB_PAD"]) if "AB_PAD" in os.environ else t.preferred_rank_stride(n)
NS = int(os.environ.get("AB_SETS", "8"))
sets = [torch.randint(0x3F80, 0x42C8, (P, stride), dtype=torch.int16, device="cuda") for _ in range(NS)]
algo = {"swing": t.SWING, "recdub": t.RECDUB}[os.environ.get("AB_ALGO", "swing")]
exec_mode = t.EXEC_STEPS if os.environ.get("AB_EXEC") == "steps" else t.EXEC_FUSED
plan = t.Plan(algo, variant, SIDE, n, P, exec_mode)
ws = torch.empty(max(plan.workspace_bytes, 16), dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for i in range(10):
        plan.execute(sets[i % NS].data_ptr(), stride, ws.data_ptr(), s)
torch.cuda.synchronize()
eager = os.environ.get("AB_EAGER") == "1"   # plain launches (PMC passes)
if not eager:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(steps):
            plan.execute(sets[i % NS].data_ptr(), stride, ws.data_ptr(), s)
    torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
with torch.cuda.stream(s):
    if eager:
        for i in range(steps):
            plan.execute(sets[i % NS].data_ptr(), stride, ws.data_ptr(), s)
    else:
        g.replay()
e1.record(s)
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / steps * 1e3
alg = 2 * P * n * 2
print(json.dumps({"variant": sys.argv[1], "P": P, "exec": os.environ.get("AB_EXEC", "fused"), "lib": os.environ.get("ALLRED_LIB_PATH", ""), "algo": os.environ.get("AB_ALGO", "swing"), "bytes_per_rank": n * 2, "us": round(us, 3),
                  "hbm_GBps": round(alg / us / 1e3, 1), "env": {k: v for k, v in os.environ.items()
                                                               if k.startswith(("ALLRED_", "AB_"))}}))
plan.close()
