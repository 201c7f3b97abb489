"""How the per-step time of the config-2 fused pass depends on the timing
method (bench.py's contract: K timed steps bracketed by synchronize):
  graph   R back-to-back replays of a K-step HIP graph, median replay / K
  eager   K eager launches behind a spin kernel that covers host submission
  graphk  one replay of a K-step graph behind the spin kernel
for K in {20, 200}.  Prints one JSON line per (method, K).
  python tools/timing_probe.py
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(device=dev)
    stride = t.preferred_rank_stride(bench.ELEMS)
    sets = [torch.empty((bench.RANKS, stride), dtype=torch.int16, device=dev) for _ in range(32)]
    for i, s in enumerate(sets):
        bench.fill_reference_convention(s[:, :bench.ELEMS], 1000 + i)
    plan = t.Plan(t.SWING, t.BO, bench.SIDE, bench.ELEMS, bench.RANKS, t.EXEC_FUSED)

    def step(i):
        plan.execute(sets[i % 32].data_ptr(), stride, None, stream)

    def warm():
        with torch.cuda.stream(stream):
            for i in range(4000):
                step(i)
        torch.cuda.synchronize()

    for K in (20, 200):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for i in range(K):
                step(i)
        torch.cuda.synchronize()
        # (events recorded inside a capture cannot be timed here: elapsed_time on
        # them fails with hipErrorInvalidHandle on ROCm 7.2 / torch 2.10)
        for method in ("graph", "eager", "graphk", "eager", "graph"):
            res = []
            for rep in range(5):
                warm()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
                with torch.cuda.stream(stream):
                    torch.cuda._sleep(max(200000, K * 15000))
                ev[0].record(stream)
                with torch.cuda.stream(stream):
                    if method == "graph":
                        for r in range(5):
                            g.replay()
                            ev[r + 1].record(stream)
                    elif method == "graphk":
                        g.replay()
                        ev[1].record(stream)
                    else:
                        for i in range(K):
                            step(i)
                        ev[1].record(stream)
                torch.cuda.synchronize()
                if method == "graph":
                    res.append(statistics.median(ev[r].elapsed_time(ev[r + 1]) for r in range(5)) / K)
                else:
                    res.append(ev[0].elapsed_time(ev[1]) / K)
            print(json.dumps({"method": method, "K": K, "us_per_step": [round(x * 1e3, 3) for x in res]}), flush=True)


if __name__ == "__main__":
    main()
