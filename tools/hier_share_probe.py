#!/usr/bin/env python3
"""W processes sharing ONE GPU run the hierarchical step (64 virtual ranks x 640 kB
each, peer windows IPC-mapped between the processes) in a given form, arms
interleaved; per arm the max over ranks of the per-step time.  A rehearsal of
the N > 1 path's hand-offs and polls (the GPU's HBM and CUs are shared W ways,
so the numbers compare arms, they are no N > 1 figure).
  python tools/hier_share_probe.py [world] [steps] [rounds]
Arms: ws (k_hier_ws), x2 (k_hier_x2).  The JSON line is the last line of stdout (gloo
prints its own lines there).  (Round 5: an idle-poll backoff of k_hier_ws's writing waves
measured no better, W = 2 / 4: 46.97 / 94.12 vs 46.80 / 93.15 us; not kept.)"""
import json
import os
import socket
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARMS = {"ws": {}, "x2": {}}


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, steps, rounds, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import tenstorrentallreduce_amd as t
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, n = 64, 327680
    peer = t.Peer(world, rank, 0, 2 * n)
    handles = [None] * world
    dist.all_gather_object(handles, peer.handle())
    peer.connect(handles)
    peer.set_max_groups(256 // world)   # every process's grid resident on the shared GPU
    sets = [torch.randint(0x3F80, 0x42C8, (P, n), dtype=torch.int16, device="cuda") for _ in range(4)]
    ws = torch.empty(n, dtype=torch.int16, device="cuda")
    s = torch.cuda.Stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {k: [] for k in ARMS}

    def run(name, k):
        if name == "x2":
            for i in range(k):
                peer.allreduce_pipelined2(sets[i % 4].data_ptr(), n, s)
            peer.allreduce_pipelined2(None, n, s)
        else:
            for i in range(k):
                peer.allreduce(sets[i % 4].data_ptr(), n, s, P, 8, t.SWING, ws.data_ptr())

    for _ in range(rounds):
        for name, knobs in ARMS.items():
            for key, v in knobs.items():
                t.tune(key, v)
            peer.set_hier_ll(1)
            run(name, 3)
            torch.cuda.synchronize()
            dist.barrier()
            e0.record(s)
            run(name, steps)
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / steps
            got = [None] * world
            dist.all_gather_object(got, us)
            res[name].append(round(max(got), 2))
            dist.barrier()
    status = peer.status()
    peer.close()
    dist.destroy_process_group()
    q.put((rank, res, status))


def main():
    import torch.multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, steps, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    r0 = [r for r in out if r[0] == 0][0][1]
    print(json.dumps({"world": world, "steps": steps, "us_per_step_max_over_ranks": r0,
                      "median": {k: statistics.median(v) for k, v in r0.items()},
                      "peer_status": [o[2] for o in out]}))


if __name__ == "__main__":
    main()
