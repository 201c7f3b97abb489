"""Tile-sum microbench: dst += src over n bf16, 64 kB .. 1 GiB.

Algorithmic bytes = 3 * n * 2 (read dst, read src, write dst); HIP events on
the launch stream; rotating buffer pairs so large sizes stream from HBM.
Prints one JSON line per size plus a summary line.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import tenstorrentallreduce_amd as t  # noqa: E402

HBM_PEAK = 8000.0


def main():
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(device=dev)
    sizes = [64 << 10, 1 << 20, 16 << 20, 64 << 20, 256 << 20, 1 << 30]
    rows = []
    for nbytes in sizes:
        n = nbytes // 2
        pairs = max(1, min(8, (1 << 30) // nbytes))  # >= 1 GiB of distinct data when possible
        bufs = [(torch.ones(n, dtype=torch.bfloat16, device=dev), torch.ones(n, dtype=torch.bfloat16, device=dev))
                for _ in range(pairs)]
        reps = max(20, min(2000, (4 << 30) // (3 * nbytes)))
        with torch.cuda.stream(stream):
            for i in range(5):
                d, s = bufs[i % pairs]
                t.bf16_add(d.data_ptr(), s.data_ptr(), n, stream)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(reps):
            d, s = bufs[i % pairs]
            t.bf16_add(d.data_ptr(), s.data_ptr(), n, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        gbps = 3 * nbytes / (us * 1e-6) / 1e9
        row = {"bytes": nbytes, "reps": reps, "us": round(us, 3), "GBps": round(gbps, 1),
               "frac": round(gbps / HBM_PEAK, 4), "resident_set_MiB": pairs * 2 * nbytes >> 20}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del bufs
        torch.cuda.empty_cache()
    print(json.dumps({"tilesum_best_frac": max(r["frac"] for r in rows if r["bytes"] >= (256 << 20))}))


if __name__ == "__main__":
    main()
