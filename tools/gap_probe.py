#!/usr/bin/env python3
"""Does a live peer set (its uncached hipExtMallocWithFlags windows / flag area)
change the per-launch cost of OTHER kernels?  The round-6 trace of the N = 1
bench showed 0.9 us between consecutive k_hier_ws dispatches against 0.2 us
between k_tree_lds_lag / k_steps_reg ones (tools/trace_gaps.py), and only the
hierarchical kernels run while a peer set exists.  Phases, each the fused
config-2 pass timed like the bench (behind a spin kernel, R repetitions of K
eager launches, median): before any peer, with a one-rank peer set of the
bench's size, then its k_hier_ws step, after closing it, with a small peer
set.  Run plain and under rocprofv3 --kernel-trace (then tools/trace_gaps.py).

  python tools/gap_probe.py [steps] [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import tenstorrentallreduce_amd as t  # noqa: E402
from bench import ELEMS, RANKS, SIDE, fill_reference_convention, timed_eager  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(device=dev)
stride = t.preferred_rank_stride(ELEMS)
sets = [torch.empty((RANKS, stride), dtype=torch.int16, device=dev) for _ in range(32)]
for i, x in enumerate(sets):
    fill_reference_convention(x[:, :ELEMS], 1000 + i)
hsets = [torch.randint(0x3F80, 0x42C8, (RANKS, ELEMS), dtype=torch.int16, device=dev) for _ in range(8)]
ws = torch.empty(ELEMS, dtype=torch.int16, device=dev)
plan = t.Plan(t.SWING, t.BO, SIDE, ELEMS, RANKS, t.EXEC_FUSED)
torch.cuda.synchronize()


def fused():
    for i in range(steps):
        plan.execute(sets[i % 32].data_ptr(), stride, None, stream)


def phase(name, run):
    with torch.cuda.stream(stream):
        for _ in range(3):
            run()
    torch.cuda.synchronize()
    r = timed_eager(stream, run, steps, reps)
    out[name] = {k: r[k] for k in ("us_per_step", "us_per_step_reps", "spread_us", "host_submit_us_per_step",
                                   "spin_covered_submission")}
    print(name, out[name]["us_per_step"], file=sys.stderr, flush=True)


out = {"steps": steps, "reps": reps}
phase("fused_no_peer", fused)
peer = t.Peer(1, 0, 0, 2 * ELEMS)
peer.connect([peer.handle()])


def hier():
    for i in range(steps):
        peer.allreduce(hsets[i % 8].data_ptr(), ELEMS, stream, RANKS, SIDE, t.SWING, ws.data_ptr())


phase("fused_peer_live", fused)
phase("hier_ws_peer_live", hier)
phase("fused_peer_live_after_hier", fused)
peer.close()
torch.cuda.synchronize()
phase("fused_peer_closed", fused)
small = t.Peer(1, 0, 0, 16384)
small.connect([small.handle()])
phase("fused_small_peer_live", fused)
small.close()
phase("fused_end", fused)
plan.close()
print(json.dumps(out))
