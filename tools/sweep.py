"""Size sweep of the virtual-rank engine on one GPU (device-resident, HIP events).

The reference's timing_taker.py sweep (python/timing_taker.py:121-126):
  LO  sizes 1..320 tiles (2 kB .. 640 kB per rank), Swing and RecDub
  BO / mem sizes 1..5 tiles per block (128 kB .. 640 kB per rank)
on the 8x8 grid, every variant in both execution forms (schedule steps /
fused).  One JSON line per point: us per allreduce (median of rounds), GB/s
of rank bytes, HBM GB/s of the form's algorithmic traffic.  From 128 kB per
rank the rotating bucket sets total >= 1 GiB (cold HBM); below, 4 warm sets
(the latency regime).  The timed launches are queued behind a spin kernel, so
small buckets measure back-to-back GPU time, not the host's launch rate.
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import tenstorrentallreduce_amd as t  # noqa: E402

SIDE, RANKS = 8, 64
SPIN = int(os.environ.get("SPIN_CYCLES", "20000000"))


def alg_bytes(variant, exec_mode, n, launches, steps=6):
    P, b = RANKS, 2
    if exec_mode == t.EXEC_FUSED or (variant != t.MEM and launches == 1):
        return 2 * P * n * b   # one HBM pass (the round-2 schedule form reads and writes every rank row once)
    # round 1's one launch per step (allred_tune_set("steps_form", 1))
    if variant == t.BO:  # RS: 3 x (P * n/2^(k+1)) per step; AG: 2 x same
        return sum(5 * P * (n >> (k + 1)) * b for k in range(steps))
    if variant == t.LO:
        return steps * 3 * P * n * b
    return (P * n + n) * b + (n + P * n) * b  # mem: reduce (read all, write dst) + broadcast


def time_plan(variant, algo, exec_mode, n, reps, rounds=5):
    dev = torch.device("cuda:0")
    stride = t.preferred_rank_stride(n)
    # bandwidth regime (>= 128 kB per rank): rotating sets of >= 1 GiB in all (cold HBM, the
    # 256 MiB MALL cannot hold them); latency regime (smaller): 4 sets, warm as in a loop
    # re-reducing one small bucket
    set_bytes = RANKS * stride * 2
    sets = 4 if n * 2 < (128 << 10) else max(4, -(-(1 << 30) // set_bytes))
    bufs = [torch.full((RANKS, stride), 0x3F80, dtype=torch.int16, device=dev) for _ in range(sets)]
    plan = t.Plan(algo, variant, SIDE, n, RANKS, exec_mode)
    ws = torch.empty(max(plan.workspace_bytes, 16), dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(rounds):
        for i in range(3):
            plan.execute(bufs[i % sets].data_ptr(), stride, ws.data_ptr(), st)
        with torch.cuda.stream(st):   # the GPU busy while the host queues the reps: GPU time, not launch rate
            torch.cuda._sleep(SPIN)
        e0.record(st)
        for i in range(reps):
            plan.execute(bufs[i % sets].data_ptr(), stride, ws.data_ptr(), st)
        e1.record(st)
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / reps)
    launches = plan.launches
    plan.close()
    return statistics.median(res), launches


def main():
    names = {t.BO: "BO", t.LO: "LO", t.MEM: "MEM"}
    points = []
    for tiles in (1, 2, 4, 8, 16, 32, 64, 128, 192, 256, 320):
        points.append((t.LO, t.normalize_tiles(tiles, RANKS, False), tiles))
    for tiles in (1, 2, 3, 4, 5):
        points.append((t.BO, t.normalize_tiles(tiles, RANKS, True), tiles))
        points.append((t.MEM, t.normalize_tiles(tiles, RANKS, True), tiles))
    for variant, nt, tiles_arg in points:
        n = nt * 1024
        for algo in (t.SWING, t.RECDUB):
            if variant == t.MEM and algo == t.RECDUB:
                continue
            for exec_mode in (t.EXEC_STEPS, t.EXEC_FUSED):
                reps = 200 if n * RANKS * 2 < (64 << 20) else 50
                us, launches = time_plan(variant, algo, exec_mode, n, reps)
                ab = alg_bytes(variant, exec_mode, n, launches)
                print(json.dumps({
                    "variant": names[variant], "algo": "swing" if algo == t.SWING else "recdub",
                    "exec": "fused" if exec_mode == t.EXEC_FUSED else "steps", "tiles_arg": tiles_arg,
                    "bytes_per_rank": n * 2, "launches": launches, "us": round(us, 3),
                    "rank_GBps": round(RANKS * n * 2 / (us * 1e-6) / 1e9, 2),
                    "hbm_GBps": round(ab / (us * 1e-6) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
