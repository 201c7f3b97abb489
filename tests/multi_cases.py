"""Shared by tests/test_multi_host.py (CPU, host-twin backend) and
tests/test_gpu_multi.py (GPU, peer-window backend with every group on one
device): the INTEGRATION.md §1 invocations of the reference executables
across G GPUs, and the oracle's composition of what allred_run across G GPUs
must produce for them.

The composition follows the plan (allred_multi_plan_build):
- FLAT (one rank per GPU): the reference's own (side, total) schedule over the
  GPUs — oracle.allreduce(variant) of the rank vectors;
- HIER (L ranks per GPU): each GPU's partial = the tree of its local rank 0 on
  the (algo, local_side, L) sub-grid (= the LO value of local rank 0), the
  partials allreduced on the (grid_side(G), G) GPU grid with the variant, the
  GPU's result written to all its L ranks;
- LOCAL (mem_2D, G = 1): oracle mem_2D over every rank.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402  (test infrastructure: the checker)

import tenstorrentallreduce_amd as t  # noqa: E402

VNAME = {t.BO: "bo", t.LO: "lo", t.MEM: "mem"}
BIN = {t.BO: "allred_BO_2D", t.LO: "allred_LO_2D", t.MEM: "allred_mem_2D"}


def mem_side(g):
    return {1: 1, 2: 2, 4: 2, 8: 4}[g]


def invocations(g):
    """(name, program, argv without argv[0], ALLRED_NODES or None) — INTEGRATION.md §1."""
    out = [
        ("config3_recdub_bo", t.BO, ["0", "1", "4", "13", "40", "32", "0", "1"], 8),   # BASELINE config 3
        ("config2_64_ranks", t.BO, ["1", "1", "8", "13", "5", "32", "0", "1"], None),  # 64 ranks over G GPUs
        ("lo_2d_legacy", t.LO, ["1", "1", "4", "13", "4", "32"], 8),                    # allred_LO_2D
        ("mem_one_rank_per_gpu", t.MEM, ["1", "1", str(mem_side(g)), "13", "40", "32"], g),
    ]
    for tiles in (1, 4, 16, 64):   # BASELINE config 5: Swing LO 2 kB ... 128 kB
        out.append((f"config5_swing_lo_{tiles}t", t.BO, ["1", "1", "4", "13", str(tiles), "32", "0", "0"], 8))
    return out


def gf_mul(a, b, S):
    poly = {1: 0x3, 2: 0x7, 3: 0xB}[S]
    r = 0
    for i in range(S):
        if (b >> i) & 1:
            r ^= a << i
    for i in range(2 * S - 2, S - 1, -1):
        if (r >> i) & 1:
            r ^= poly << (i - S)
    return r


def channel_count(desc, n):
    """channels_for(): buckets >= 1 MiB on an XOR grid use every link, else 1."""
    if n * 2 < (1 << 20):
        return 1
    rc, s = oracle.schedule(desc.algo, desc.side_length, desc.total_nodes)
    S = s.steps
    if S < 1 or S > 3:
        return 1
    for k in range(S):
        m = s.partner[0][k]
        if any(s.partner[x][k] != (x ^ m) for x in range(desc.total_nodes)):
            return 1
    return (1 << S) - 1


def channel_allreduce(variant, algo, side, total, vecs, C):
    """The schedule over C link-spreading channels (dist.cpp slice_of / gf relabel)."""
    if C == 1:
        oracle.allreduce(variant, algo, side, vecs, total)
        return
    S = total.bit_length() - 1
    n = vecs[0].size
    unit = 8 * total
    q, rem = divmod(n // unit, C)
    start = 0
    for c in range(C):
        ln = (q + (1 if c < rem else 0)) * unit
        a = 1
        for _ in range(c):
            a = gf_mul(a, 2, S)
        lab = [gf_mul(a, r, S) for r in range(total)]
        base = [None] * total
        for r in range(total):
            base[lab[r]] = vecs[r][start:start + ln].copy()
        oracle.allreduce(variant, algo, side, base, total)
        for r in range(total):
            vecs[r][start:start + ln] = base[lab[r]]
        start += ln


def expected(plan, data):
    """Every rank's result (total, elems) for `data` (total, elems) under `plan`."""
    G, L, N = plan.gpus, plan.local_ranks, plan.total_nodes
    d = plan.desc
    acc16 = d.mem_accum == t.ACC_BF16
    out = np.empty_like(data)
    if plan.mode == t.MULTI_LOCAL:
        ranks = [r.copy() for r in data]
        oracle.allreduce("mem", d.algo, 1, ranks, N, acc16)
        return np.stack(ranks)
    if plan.mode == t.MULTI_FLAT:
        ranks = [r.copy() for r in data]
        if plan.variant == t.MEM:
            oracle.allreduce("mem", d.algo, d.side_length, ranks, N, acc16)
        else:
            channel_allreduce(VNAME[plan.variant], d.algo, d.side_length, N, ranks,
                              channel_count(d, int(plan.elems)))
        return np.stack(ranks)
    partials = []
    for g in range(G):
        loc = [r.copy() for r in data[g * L:(g + 1) * L]]
        oracle.allreduce("lo", d.local_algo, d.local_side, loc, L)   # tree of local rank 0
        partials.append(loc[0])
    channel_allreduce(VNAME[plan.variant], d.algo, d.side_length, G, partials, channel_count(d, int(plan.elems)))
    for g in range(G):
        out[g * L:(g + 1) * L] = partials[g]
    return out


def random_inputs(total, n, seed):
    rng = np.random.default_rng(seed)
    # finite bf16 in [1, 100) with random signs: rounding differs between trees
    mag = rng.integers(0x3F80, 0x42C8, (total, n)).astype(np.uint16)
    return mag | (rng.integers(0, 2, (total, n)).astype(np.uint16) << 15)


def argv_error0(argv, variant):
    """The invocation with ERROR = 0 (argv[6]): exact parity with the reference's expected value."""
    a = list(argv)
    a[5] = "0"
    return a


# ---------------------------------------------------------------- the RCCL multi-device cases
# tests/test_gpu_multidevice.py runs these on real communicators (one thread per device); their
# CPU twin, tests/test_multidevice_host.py, runs the SAME cases through the host twin of the RCCL
# program (allred_dist_allreduce_host over gloo) against the SAME expectation code, so a red case
# on the first multi-GPU box points at the product, not at the test (verdict r05 item 3).
def rccl_cases(world, big=1 << 19):
    """(variant, algo, local_ranks, channels, n): every case of tests/test_dist_host.py's gloo
    matrix at n = 8 x total x 48, then flat BO / LO x RecDub / Swing at `big` elements per rank
    with the auto channels (channels 0: every link from 1 MiB on)."""
    import test_dist_host as tdh
    side, total = tdh.GRIDS[world]
    n = 8 * total * 16 * 3
    out = [(v, a, loc, ch, n) for (v, a, loc, ch) in tdh.cases(world)]
    for v in ("bo", "lo"):
        for a in (t.RECDUB, t.SWING):
            out.append((v, a, 1, 0, big))
    return out


def rccl_case_desc(world, variant, algo, local, chans, n):
    import test_dist_host as tdh
    side, total = tdh.GRIDS[world]
    return t.dist_desc(algo, t.BO if variant == "bo" else t.LO, 1 if algo >= 2 else side, total, n,
                       local_ranks=local, local_side=2, local_algo=t.SWING, channels=chans)


def rccl_case_inputs(world, local, n, ci, rep):
    """the per-rank inputs of case ci, repetition rep (identical on every rank: same seed)"""
    import test_dist_host as tdh
    return tdh.inputs(world, local, n, seed=5000 * world + 10 * ci + rep)


def rccl_case_expected(world, variant, algo, local, chans, n, data):
    """every rank's expected bucket (local rows concatenated) of a rccl_cases() case"""
    import test_dist_host as tdh
    desc = rccl_case_desc(world, variant, algo, local, chans, n)
    C = chans if chans else channel_count(desc, n)
    return [np.concatenate(x) for x in tdh.expected(variant, algo, world, local, data, C)]


def rccl_mem_inputs(world, acc, n):
    return [np.random.default_rng(77 * world + acc + g).integers(0x3F80, 0x42C8, n).astype(np.uint16)
            for g in range(world)]


def rccl_mem_expected(world, acc, data):
    """mem_2D over RCCL (local_ranks 1): the oracle's allred_mem_2D restatement, fp32 or the
    reference's bf16 accumulation"""
    import test_dist_host as tdh
    side, total = tdh.GRIDS[world]
    want = [d.copy() for d in data]
    oracle.allreduce("mem", t.SWING, side, want, total, acc == t.ACC_BF16)
    return want


def pipelined_inputs(world, n, local=64, K=3):
    """data[k][g]: bucket k of GPU g, `local` rank rows of n elements"""
    return [[np.random.default_rng(9000 + 97 * k + g).integers(0x3F80, 0x42C8, (local, n)).astype(np.uint16)
             for g in range(world)] for k in range(K)]


def pipelined_expected(world, n, data_k, local=64):
    """one bucket of the rccl_x transport (allred_dist_allreduce_pipelined with 64 local ranks):
    every GPU's partial = the oracle's tree of its local rank 0 (8x8 Swing), the partials
    allreduced by the 2D Swing BO over the GPU grid (link-spreading channels where the bucket
    takes them), the result in all 64 rows -> expected partial of every GPU"""
    import test_dist_host as tdh
    side, total = tdh.GRIDS[world]
    desc = t.dist_desc(t.SWING, t.BO, side, total, n, local_ranks=local, local_side=8, local_algo=t.SWING)
    partials = []
    for g in range(world):
        loc = [x.copy() for x in data_k[g]]
        oracle.allreduce("lo", t.SWING, 8, loc, local)   # tree of local rank 0
        partials.append(loc[0])
    channel_allreduce("bo", t.SWING, side, total, partials, channel_count(desc, n))
    return partials


def config4_ints(n, r, dev):
    """BASELINE config 4's data for rank r: small integers 0..7 in bf16 (a per-element hash of
    (e, r)), so every partial sum of up to 8 ranks is exact whatever the reduction order"""
    import torch
    e = torch.arange(n, dtype=torch.int64, device=dev)
    return (((e * 2654435761 + r * 40503) >> 13) & 7).to(torch.bfloat16)


def config4_exact(n, world, dev):
    """the exact sum of the world's config4_ints, fp32"""
    import torch
    acc = torch.zeros(n, dtype=torch.float32, device=dev)
    for r in range(world):
        acc += config4_ints(n, r, dev).float()
    return acc
