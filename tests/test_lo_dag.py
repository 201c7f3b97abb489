"""The fused LO pass's DAG of distinct sums (allred_lo_dag, the table
k_butterfly_lds64_pipe reads), checked on the CPU: evaluating the table the
way the kernel does — per step all reads, then all writes, rank r's result in
row fin[r] — reproduces the oracle's per-rank LO butterfly
(allred_BO_2D/kernels/dataflow_kernel.cpp:19-29 over the schedule of
allred_helper.cpp:145-191) bit for bit, and the placed table's reads are
bank-conflict free."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle
import tenstorrentallreduce_amd as t
from tenstorrentallreduce_amd import _lib

DAG_BYTES = 456 + 32 * 6


def lo_dag(algo, side=8, total=64):
    buf = (C.c_uint8 * DAG_BYTES)()
    conflicts = C.c_int(-1)
    n = _lib.lib.allred_lo_dag(algo, side, total, buf, DAG_BYTES, C.byref(conflicts))
    assert n >= 0, n
    return np.frombuffer(bytes(buf), dtype=np.uint8)[:n], conflicts.value


def bf16_add(a, b):
    """fp32 add of two bf16 arrays, rounded to nearest even (v_cvt_pk_bf16_f32)."""
    s = ((a.astype(np.uint32) << 16).view(np.float32) + (b.astype(np.uint32) << 16).view(np.float32))
    u = s.view(np.uint32)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def evaluate(dag, leaves):
    """The kernel's DAG pass over a [64, n] tile of leaves."""
    tile = leaves.copy()
    steps = int(np.count_nonzero(dag[448:454]))
    for k in range(steps):
        nodes = [(int(dag[k * 64 + 2 * s]), int(dag[k * 64 + 2 * s + 1]), int(dag[456 + 32 * k + s]))
                 for s in range(32) if dag[k * 64 + 2 * s] != 0xFF]
        assert len(nodes) == dag[448 + k]
        outs = [bf16_add(tile[a], tile[b]) for a, b, _ in nodes]   # every read before any write
        rows = [d for _, _, d in nodes]
        assert len(set(rows)) == len(rows), "two nodes of one step share a row"
        for d, v in zip(rows, outs):
            tile[d] = v
    if steps:
        assert int(dag[384:448].max()) < int(dag[448 + steps - 1]), "final rows are the last step's 0..d_last-1"
    return tile[dag[384:448].astype(np.int64)]


@pytest.mark.parametrize("algo", [t.SWING, t.RECDUB])
@pytest.mark.parametrize("seed", [13, -1])
def test_dag_matches_oracle_lo(algo, seed):
    dag, conflicts = lo_dag(algo)
    assert dag.size == DAG_BYTES
    assert conflicts == 0
    n = 256
    if seed < 0:   # the reference's all-ones known answer
        ranks = [np.full(n, 0x3F80, dtype=np.uint16) for _ in range(64)]
    else:          # a distinct vector per rank, so that a wrong operand row shows
        ranks = [oracle.random_bf16_vector(2 * n, seed + r).view(np.uint16).copy() for r in range(64)]
    leaves = np.stack(ranks)
    want = [r.copy() for r in ranks]
    oracle.allreduce("lo", algo, 8, want)
    got = evaluate(dag, leaves)
    np.testing.assert_array_equal(got, np.stack(want))


def test_swing_dag_shape_and_placement():
    dag, conflicts = lo_dag(t.SWING)
    assert list(dag[448:454]) == [32, 16, 16, 16, 8, 4]   # 92 distinct sums per column
    assert conflicts == 0
    with t.tuned(lo_dag_place=0):
        unplaced, c0 = lo_dag(t.SWING)
    assert c0 == 92   # first-appearance rows and slots: one extra cycle per read group and item on average
    np.testing.assert_array_equal(evaluate(unplaced, np.arange(64 * 8, dtype=np.uint16).reshape(64, 8) + 0x3F80),
                                  evaluate(dag, np.arange(64 * 8, dtype=np.uint16).reshape(64, 8) + 0x3F80))


def test_no_dag_off_64_ranks():
    assert lo_dag(t.SWING, 4, 16)[0].size == 0
    assert lo_dag(t.SWING, 2, 4)[0].size == 0


# ------------------------------------------------------------------ register DAG (build-time)
INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tenstorrentallreduce_amd", "build",
                   "lo_dag_gen.inc")


def generated_dags():
    """The DAGs csrc/gen_lo_dag.cpp wrote into build/lo_dag_gen.inc at build time
    (k_lo_dag_reg's compile-time tables), parsed back: {(algo, side, total): dict}."""
    import re
    text = open(INC).read()
    out = {}
    for m in re.finditer(r"struct (LoDag\d+) \{[^\n]*\n(.*?)\n\};", text, re.S):
        body = m.group(2)
        arr = {k: [int(x) for x in v.replace("\n", " ").split(",")]
               for k, v in re.findall(r"static constexpr int (\w+)\[\d+\] = \{(.*?)\};", body, re.S)}
        hdr = dict(re.findall(r"(\w+) = (\d+)", body.split("\n")[0]))
        arr.update({k: int(v) for k, v in hdr.items()})
        out[m.group(1)] = arr
    keys = {}
    for name, algo, side, total in re.findall(r"X\((LoDag\d+), (\d+), (\d+), (\d+)\)", text):
        keys[(int(algo), int(side), int(total))] = out[name]
    return keys


@pytest.mark.skipif(not os.path.exists(INC), reason="build() writes the generated DAG header")
def test_register_dag_header_matches_oracle_lo():
    """Every generated DAG, evaluated the way k_lo_dag_reg does (node P + i =
    RNE(v[a[i]] + v[b[i]]), rank r gets node fnode[fin[r]]), reproduces the
    oracle's per-rank LO butterfly bit for bit; and it covers exactly the Swing
    schedules at 32 / 64 ranks whose ranks do not share one tree (8x8 and 8x4
    2D, 1D at 32; 1D at 64 has 16 distinct finals and keeps the LDS DAG pass)."""
    dags = generated_dags()
    assert set(dags) == {(t.SWING, 8, 64), (t.SWING, 8, 32), (t.SWING_1D, 1, 32)}
    assert dags[(t.SWING, 8, 64)]["N"] == 92 and dags[(t.SWING, 8, 64)]["F"] == 4
    rng = np.random.default_rng(7)
    for (algo, side, total), d in dags.items():
        P, N, F = d["P"], d["N"], d["F"]
        assert P == total and len(d["a"]) == len(d["b"]) == N and len(d["fnode"]) == F and len(d["fin"]) == P
        n = 512
        ranks = [(rng.integers(0, 0x7000, n) | (rng.integers(0, 2, n) << 15)).astype(np.uint16) for _ in range(P)]
        v = list(ranks)
        for i in range(N):
            assert d["a"][i] < P + i and d["b"][i] < P + i, "operands precede the node"
            v.append(bf16_add(v[d["a"][i]], v[d["b"][i]]))
        got = np.stack([v[d["fnode"][d["fin"][r]]] for r in range(P)])
        want = [r.copy() for r in ranks]
        oracle.allreduce("lo", algo, side, want, total)
        assert (got == np.stack(want)).all(), (algo, side, total)
