"""Times allred_peer create / handle / connect for several window sizes with
`world` processes on one GPU (IPC handles exchanged over gloo).  Diagnostic for
the bench's 1 GiB peer windows; prints one line per stage to stderr.

    python tools/peer_open_probe.py --world 2 --sizes 1048576,67108864,536870912
    python tools/peer_open_probe.py --world 4 --keep --sizes 268435456,268435456
"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def log(rank, msg):
    print(f"[probe r{rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def worker(rank, world, sizes, port, keep):
    import tenstorrentallreduce_amd as t
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    kept = []
    for n in sizes:
        t0 = time.perf_counter()
        peer = t.Peer(world, rank, 0, n)
        log(rank, f"max_elems {n}: create {time.perf_counter() - t0:.3f}s")
        t0 = time.perf_counter()
        h = peer.handle()
        log(rank, f"max_elems {n}: handle {time.perf_counter() - t0:.3f}s")
        handles = [None] * world
        dist.all_gather_object(handles, h)
        t0 = time.perf_counter()
        peer.connect(handles)
        log(rank, f"max_elems {n}: connect {time.perf_counter() - t0:.3f}s")
        dist.barrier()
        if keep:
            kept.append(peer)
        else:
            peer.close()
        dist.barrier()
    for peer in kept:
        peer.close()
    log(rank, "done")
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--sizes", default="1048576,67108864,536870912")
    ap.add_argument("--keep", action="store_true", help="keep every window open until the end")
    args = ap.parse_args()
    sizes = [int(s) for s in args.sizes.split(",")]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=worker, args=(r, args.world, sizes, 29650, args.keep)) for r in range(args.world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
    sys.exit(max(abs(p.exitcode or 0) for p in procs))


if __name__ == "__main__":
    main()
