#!/usr/bin/env python3
"""Host-staged end-to-end time of BASELINE config 2 through allred_run (the
reference CLI's path: buckets start and end in pinned host memory) for a set of
ALLRED_E2E / ALLRED_E2E_CHUNKS arms, interleaved, median of R runs each.
  python tools/e2e_probe.py [R]   -> one JSON line"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tenstorrentallreduce_amd as t  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 5
WARM = os.environ.get("E2E_WARM") == "1"   # torch initialised + ~50 ms of GPU work before every run
if WARM:
    import torch
    _a = torch.randn(4096, 4096, device="cuda")


def warm():
    if WARM:
        for _ in range(20):
            _a @ _a
        torch.cuda.synchronize()
ARMS = {"zerocopy": {"ALLRED_E2E": "zerocopy"}, "dma_default": {"ALLRED_E2E": "dma"},
        "dma_1": {"ALLRED_E2E": "dma", "ALLRED_E2E_CHUNKS": "1"}, "dma_8": {"ALLRED_E2E": "dma", "ALLRED_E2E_CHUNKS": "8"},
        "dma_16": {"ALLRED_E2E": "dma", "ALLRED_E2E_CHUNKS": "16"}, "dma_32": {"ALLRED_E2E": "dma", "ALLRED_E2E_CHUNKS": "32"}}
argv = ["allred_BO_2D", "1", "1", "8", "13", "5", "32", "0", "1"]
res = {k: [] for k in ARMS}
bad = 0
for _ in range(R):
    for name, env in ARMS.items():
        old = {k: os.environ.get(k) for k in ("ALLRED_E2E", "ALLRED_E2E_CHUNKS")}
        for k in old:
            os.environ.pop(k, None)
        os.environ.update(env)
        warm()
        rep = t.run(argv, t.BO, False, t.EXEC_FUSED)
        bad += int(rep.mismatches)
        res[name].append(round(rep.e2e_seconds * 1e3, 4))
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
print(json.dumps({"e2e_ms": res, "median": {k: statistics.median(v) for k, v in res.items()}, "mismatches": bad, "warm": WARM,
                  "bytes_each_way": 64 * 655360}))
