"""The schedule form's step programs (allred_steps_program: the tables
k_steps_reg reads) evaluated on the CPU the way the kernel runs them — step
0 sums pairs of staged rank rows into compact rows (every read before any
write), BO's later phases add / copy among those rows, LO's later steps add
the row kept in the lane's register to the other operand row — against the
oracle's per-rank BO and LO programs (allred_BO_2D/kernels/dataflow_kernel.cpp
:152-267, allred_LOO_2D/kernels/dataflow_kernel.cpp:127-175), bit for bit.
Also pins the LO table's matching property: in every step after the first,
pair x's first operand is row x (the value the lane already holds)."""
import ctypes as C

import numpy as np
import pytest

import oracle
import tenstorrentallreduce_amd as t
from tenstorrentallreduce_amd import _lib

GRIDS = [(2, 2), (2, 4), (4, 8), (4, 16), (8, 32), (8, 64)]


def program(algo, variant, side, total):
    cap = max(total * 256, 2 * (total // 2) * 6 + total)
    buf = (C.c_uint8 * cap)()
    n = _lib.lib.allred_steps_program(algo, variant, side, total, buf, cap)
    assert n > 0, n
    return np.frombuffer(bytes(buf), dtype=np.uint8)[:n].astype(np.int64)


def bf16_add(a, b):
    s = ((a.astype(np.uint32) << 16).view(np.float32) + (b.astype(np.uint32) << 16).view(np.float32))
    u = s.view(np.uint32)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def run_bo(tab, total, block):
    """the BO schedule form (k_steps_reg<P, true>) on one block's rank rows ([total, cols])."""
    H, S = total // 2, total.bit_length() - 1
    rows = block.copy()
    p0 = tab[:2 * H].reshape(H, 2)
    new = [bf16_add(rows[a], rows[b]) for a, b in p0]   # every read before any write
    for x in range(H):
        rows[x] = new[x]
    e = 2 * H
    for ph in range(1, 2 * S - 1):
        rs = ph < S
        k = ph if rs else 2 * S - 1 - ph
        for x in range(total >> (k + 1)):
            a, c = tab[e + 2 * x], tab[e + 2 * x + 1]
            rows[a] = bf16_add(rows[a], rows[c]) if rs else rows[c].copy()
        e += 2 * (total >> (k + 1))
    return np.stack([rows[tab[e + r]] for r in range(total)])


def run_lo(tab, total, ranks):
    H, S = total // 2, total.bit_length() - 1
    rows = ranks.copy()
    p0 = tab[:2 * H].reshape(H, 2)
    val = [bf16_add(rows[a], rows[b]) for a, b in p0]
    for x in range(H):
        rows[x] = val[x]
    e = 2 * H
    for _ in range(1, S):
        step = tab[e:e + 2 * H].reshape(H, 2)
        assert (step[:, 0] == np.arange(H)).all(), "pair x keeps row x in its register"
        oth = [rows[c].copy() for _, c in step]
        for x in range(H):
            val[x] = bf16_add(val[x], oth[x])
            rows[x] = val[x]
        e += 2 * H
    return np.stack([rows[tab[e + r]] for r in range(total)])


@pytest.mark.parametrize("algo", [t.SWING, t.RECDUB])
@pytest.mark.parametrize("grid", GRIDS)
def test_bo_program_matches_oracle(grid, algo):
    side, total = grid
    tab = program(algo, t.BO, side, total)
    assert tab.size == total * 256
    n = total * 16
    rng = np.random.default_rng(5 + total + algo)
    ranks = [rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(total)]
    want = [r.copy() for r in ranks]
    oracle.allreduce("bo", algo, side, want, total)
    blk = n // total
    got = np.zeros((total, n), dtype=np.uint16)
    stacked = np.stack(ranks)
    for b in range(total):
        got[:, b * blk:(b + 1) * blk] = run_bo(tab[b * 256:(b + 1) * 256], total, stacked[:, b * blk:(b + 1) * blk])
    assert (got == np.stack(want)).all()


def run_bo_reg(tab, pairs, total, block):
    """k_steps_reg<P, true> on one block's rank rows: step 0 from the block-independent
    pairs (lower, higher rank) as the loads see them, holder first, into the holder's row;
    then the same phases and result rows as the pipe table."""
    H, S = total // 2, total.bit_length() - 1
    rows = np.zeros_like(block)
    for u in range(H):
        x, swap = tab[u] & 127, tab[u] >> 7
        a, b = block[pairs[2 * u]], block[pairs[2 * u + 1]]
        rows[x] = bf16_add(b, a) if swap else bf16_add(a, b)
    e = 2 * H
    for ph in range(1, 2 * S - 1):
        rs = ph < S
        k = ph if rs else 2 * S - 1 - ph
        for x in range(total >> (k + 1)):
            a, c = tab[e + 2 * x], tab[e + 2 * x + 1]
            rows[a] = bf16_add(rows[a], rows[c]) if rs else rows[c].copy()
        e += 2 * (total >> (k + 1))
    return np.stack([rows[tab[e + r]] for r in range(total)])


@pytest.mark.parametrize("algo", [t.SWING, t.RECDUB])
@pytest.mark.parametrize("grid", GRIDS)
def test_bo_register_program_matches_oracle(grid, algo):
    """The program the register-staged schedule form loads (ALLRED_STEPS_REG): the step-0
    pairs are the same for every block (each pair once, lower rank first), every block
    maps each pair to one distinct holder row, and evaluating it bit-matches the oracle."""
    side, total = grid
    H = total // 2
    cap = total * 256 + total
    buf = (C.c_uint8 * cap)()
    n = _lib.lib.allred_steps_program(algo, t.BO | _lib.STEPS_REG, side, total, buf, cap)
    assert n == total * 256 + total, n
    prog = np.frombuffer(bytes(buf), dtype=np.uint8)[:n].astype(np.int64)
    pairs = prog[total * 256:]
    assert sorted(pairs.tolist()) == list(range(total))             # every rank in exactly one pair
    assert all(pairs[2 * u] < pairs[2 * u + 1] for u in range(H))
    pipe = program(algo, t.BO, side, total)
    rng = np.random.default_rng(11 + total + algo)
    n_el = total * 16
    ranks = [rng.integers(0x3F80, 0x42C8, n_el).astype(np.uint16) for _ in range(total)]
    want = [r.copy() for r in ranks]
    oracle.allreduce("bo", algo, side, want, total)
    blk = n_el // total
    got = np.zeros((total, n_el), dtype=np.uint16)
    stacked = np.stack(ranks)
    for b in range(total):
        tab = prog[b * 256:(b + 1) * 256]
        assert sorted((tab[:H] & 127).tolist()) == list(range(H))    # one holder row per pair
        assert (tab[2 * H:] == pipe[b * 256 + 2 * H:(b + 1) * 256]).all()   # phases, result rows as the pipe's
        got[:, b * blk:(b + 1) * blk] = run_bo_reg(tab, pairs, total, stacked[:, b * blk:(b + 1) * blk])
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("algo,grid", [(a, g) for a in (t.SWING, t.RECDUB) for g in GRIDS] +
                         [(t.SWING_1D, (1, 16)), (t.SWING_1D, (1, 64)), (t.RECDUB_1D, (1, 32))])
def test_lo_program_matches_oracle(algo, grid):
    side, total = grid
    tab = program(algo, t.LO, side, total)
    S = total.bit_length() - 1
    assert tab.size == 2 * (total // 2) * S + total
    n = 64
    rng = np.random.default_rng(9 + total + algo)
    ranks = [rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(total)]
    want = [r.copy() for r in ranks]
    oracle.allreduce("lo", algo, side, want, total)
    got = run_lo(tab, total, np.stack(ranks))
    assert (got == np.stack(want)).all()


def test_steps_program_errors():
    buf = (C.c_uint8 * 16)()
    assert _lib.lib.allred_steps_program(t.SWING, t.BO, 8, 64, buf, 16) < 0      # too small
    assert _lib.lib.allred_steps_program(t.SWING, t.MEM, 8, 64, buf, 16) < 0     # no step program
    assert _lib.lib.allred_steps_program(t.SWING, t.BO, 8, 16, buf, 16) < 0      # invalid grid
    assert _lib.lib.allred_steps_program(t.SWING, t.BO, 1, 1, buf, 16) == 0      # one rank: nothing
