"""BASELINE configs 3 and 5 at their stated sizes, the schedule form (one
persistent launch and the per-step A/B form), its device stamps, and the
reference-faithful mem_2D accumulation — all through the C-ABI on the GPU,
bit-exact against the CPU oracle.

Config 3: 8-rank RecDub BO, 655,360 B per rank, the 4x2 grid the 8-GPU
mapping uses (allred_BO_2D.cpp:96-153 masks).  Config 5: 8-rank Swing LO at
2 / 8 / 32 / 128 kB.  On one GPU the 8 ranks are virtual (plans); the
8-process peer program over IPC windows is tests/test_gpu_peer.py
test_config3_config5_eight_processes."""
import numpy as np
import pytest

import oracle
import tenstorrentallreduce_amd as t

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"

CONFIG3_N = 327680                       # 655,360 B of bf16 per rank
CONFIG5_N = [1024, 4096, 16384, 65536]   # 2, 8, 32, 128 kB


def rand_ranks(total, n, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(total)]


def run_plan(algo, variant, side, total, ranks, exec_mode, stride=None, mem_accum=t.ACC_FP32):
    n = ranks[0].size
    stride = stride or n
    host = np.zeros((total, stride), dtype=np.uint16)
    for r in range(total):
        host[r, :n] = ranks[r]
    buf = torch.from_numpy(host.view(np.int16)).to(DEV)
    plan = t.Plan(algo, variant, side, n, total, exec_mode, mem_accum=mem_accum)
    ws = torch.empty(max(plan.workspace_bytes, 16), dtype=torch.uint8, device=DEV)
    plan.execute(buf.data_ptr(), stride, ws.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    out = buf.cpu().numpy().view(np.uint16)[:, :n]
    plan.close()
    return out


# ------------------------------------------------------------------ config 3
@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
def test_config3_recdub_bo_4x2_640kB_random(exec_mode):
    side, total = 4, 8
    ranks = rand_ranks(total, CONFIG3_N, seed=303)
    got = run_plan(t.RECDUB, t.BO, side, total, ranks, exec_mode, stride=t.preferred_rank_stride(CONFIG3_N))
    want = [r.copy() for r in ranks]
    oracle.allreduce("bo", t.RECDUB, side, want, total)
    assert np.array_equal(got, np.stack(want))
    assert (got == got[0]).all()   # BO: every rank ends with the same vector


@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
def test_config3_reference_inputs_and_check(exec_mode):
    """The reference's input convention (seeds 13/14 by x parity) and its
    ±32 check on every rank (allred_helper.cpp:18-120)."""
    side, total = 4, 8
    s0, s1, ranks = oracle.reference_inputs(side, total, CONFIG3_N, 13)
    got = run_plan(t.RECDUB, t.BO, side, total, ranks, exec_mode)
    want = [r.copy() for r in ranks]
    oracle.allreduce("bo", t.RECDUB, side, want, total)
    assert np.array_equal(got, np.stack(want))
    for r in range(total):
        assert oracle.validate(got[r].view(np.uint32), s0, s1, total, 32.0)[0] == 0


# ------------------------------------------------------------------ config 5
@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
@pytest.mark.parametrize("n", CONFIG5_N)
def test_config5_swing_lo_4x2_sweep(n, exec_mode):
    side, total = 4, 8
    ranks = rand_ranks(total, n, seed=500 + n % 1009)
    got = run_plan(t.SWING, t.LO, side, total, ranks, exec_mode)
    want = [r.copy() for r in ranks]
    oracle.allreduce("lo", t.SWING, side, want, total)
    assert np.array_equal(got, np.stack(want))


@pytest.mark.parametrize("n", CONFIG5_N)
def test_config5_reference_inputs(n):
    side, total = 4, 8
    s0, s1, ranks = oracle.reference_inputs(side, total, n, 13)
    got = run_plan(t.SWING, t.LO, side, total, ranks, t.EXEC_STEPS)
    for r in range(total):
        assert oracle.validate(got[r].view(np.uint32), s0, s1, total, 32.0)[0] == 0


# ------------------------------------------------------------------ schedule form
@pytest.mark.parametrize("steps_form,groups,tabs", [(0, 0, 3), (0, 3, 3), (0, 4, 3), (0, 5, 3), (1, 0, 3), (2, 0, 3),
                                                    (0, 0, 0), (0, 5, 1), (2, 0, 1), (0, 4, 2)])
@pytest.mark.parametrize("variant", ["bo", "lo"])
@pytest.mark.parametrize("algo,grid,n", [(t.SWING, (8, 64), 327680), (t.RECDUB, (8, 64), 327680),
                                         (t.SWING, (8, 64), 64 * 8 * 3), (t.SWING, (4, 8), 8 * 8 * 5),
                                         (t.RECDUB, (2, 2), 1024), (t.SWING_1D, (1, 16), 16 * 8 * 33),
                                         (t.SWING, (1, 1), 64), (t.SWING, (4, 8), 8 * 256 * 3),
                                         (t.SWING, (8, 32), 32 * 256 * 3), (t.RECDUB, (4, 16), 16 * 256 * 5),
                                         (t.SWING_1D, (1, 16), 16 * 256 * 2), (t.SWING, (8, 64), 1 << 20)])
def test_schedule_form_bit_exact(algo, grid, n, variant, steps_form, groups, tabs):
    """The schedule form as one persistent launch (k_steps_reg, steps_form 0:
    128-byte strips of whole 512-byte units of 8..64 ranks, step 0 from
    registers, the later steps among LDS rows; other shapes fall back to
    k_bo_steps / k_lo_steps) at the auto grid and at 3 / 4 / 5 workgroups per
    CU (steps_groups), staging only its units' programs (steps_tab, default
    1) and with the first strip's loads ahead of the staging (steps_early,
    default 1) or not (the round-3 order), with
    every unit resident at once (steps_form 2) and as
    one launch per step (steps_form 1, the round-1 kernels), on slices
    narrower than a unit (3 and 5 vectors per block), odd unit counts and at
    config-2 size, against the oracle."""
    side, total = grid
    ranks = rand_ranks(total, n, seed=7 * total + n % 97 + algo)
    with t.tuned(steps_form=steps_form, steps_groups=groups, steps_tab=tabs & 1, steps_early=tabs >> 1):
        got = run_plan(algo, {"bo": t.BO, "lo": t.LO}[variant], side, total, ranks, t.EXEC_STEPS,
                       stride=n + 64)
    want = [r.copy() for r in ranks]
    oracle.allreduce(variant, algo, side, want, total)
    assert np.array_equal(got, np.stack(want))


@pytest.mark.parametrize("cap,early", [(1, 1), (16, 1), (32, 1), (200, 1), (0, 2), (0, 0)])
@pytest.mark.parametrize("variant", ["bo", "lo"])
def test_schedule_form_capped_grids(variant, cap, early):
    """k_steps_reg at config 2 on capped grids (tune pipe_grid): a workgroup
    with 40 units stages 40 block programs (steps_tab), one with 80 or 1280
    (>= P blocks) stages every block's program instead, and 200 workgroups
    leave some with one unit fewer; the default grid with the first strip's
    loads always / never ahead of the program staging — all bit-exact against
    the oracle."""
    side, total, n = 8, 64, 327680
    ranks = rand_ranks(total, n, seed=cap + 5)
    with t.tuned(pipe_grid=cap, steps_early=early):
        got = run_plan(t.SWING, {"bo": t.BO, "lo": t.LO}[variant], side, total, ranks, t.EXEC_STEPS)
    want = [r.copy() for r in ranks]
    oracle.allreduce(variant, t.SWING, side, want, total)
    assert np.array_equal(got, np.stack(want))


@pytest.mark.parametrize("steps_form,groups", [(0, 0), (2, 0), (0, 4)])
@pytest.mark.parametrize("variant", [t.BO, t.LO])
def test_schedule_form_device_stamps(variant, steps_form, groups):
    """execute(stamps_ptr=...): every unit's start and per-step stamps
    (s_memrealtime, 100 MHz) are written and monotonic within a unit; the
    per-rank zones (allred_plan_rank_zones) open before they close, and the
    whole pass takes well under a millisecond."""
    side, total, n = 8, 64, 327680
    ranks = rand_ranks(total, n, seed=99)
    host = np.stack(ranks)
    buf = torch.from_numpy(host.view(np.int16)).to(DEV)
    with t.tuned(steps_form=steps_form, steps_groups=groups):
        plan = t.Plan(t.SWING, variant, side, n, total, t.EXEC_STEPS)
    assert plan.launches == 1 and plan.stamp_words > 0
    st = torch.zeros(plan.stamp_words, dtype=torch.int64, device=DEV)
    with t.tuned(steps_form=steps_form, steps_groups=groups):
        plan.execute(buf.data_ptr(), n, None, torch.cuda.current_stream(), stamps_ptr=st.data_ptr())
    torch.cuda.synchronize()
    stamps = st.cpu().numpy().view(np.uint64)
    per = 2 * 6 + 1 if variant == t.BO else 6 + 1
    units = stamps.reshape(-1, per)
    assert (units > 0).all()
    assert (np.diff(units.astype(np.int64), axis=1) >= 0).all()
    zs, ze = plan.rank_zones(stamps)
    assert (zs < ze).all()
    assert int(ze.max() - zs.min()) < 100_000   # < 1 ms at 100 MHz
    want = [r.copy() for r in ranks]
    oracle.allreduce("bo" if variant == t.BO else "lo", t.SWING, side, want, total)
    assert np.array_equal(buf.cpu().numpy().view(np.uint16), np.stack(want))
    plan.close()


def test_stamps_rejected_by_forms_without_them():
    plan = t.Plan(t.SWING, t.BO, 8, 64 * 8, 64, t.EXEC_FUSED)
    assert plan.stamp_words == 0
    buf = torch.zeros((64, 64 * 8), dtype=torch.int16, device=DEV)
    st = torch.zeros(16, dtype=torch.int64, device=DEV)
    with pytest.raises(t.AllredError):
        plan.execute(buf.data_ptr(), 64 * 8, None, None, stamps_ptr=st.data_ptr())
    plan.close()


# ------------------------------------------------------------------ mem_2D, the reference's bf16 accumulation
@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
@pytest.mark.parametrize("grid,n", [((2, 4), 1024 * 4), ((4, 8), 8 * 8 * 9), ((4, 16), 256 * 16 * 3),
                                    ((8, 64), 327680), ((8, 64), 64 * 8 * 5)])
def test_mem_bf16_accumulation_bit_exact(grid, n, exec_mode):
    """ALLRED_ACC_BF16: own block first, then every other rank in rank order,
    the running sum rounded to bf16 after every add — the Tensix dest with
    fp32_dest_acc_en = false (allred_helper.cpp:331-335,
    allred_mem_2D/kernels/compute_kernel.cpp:44-67) — in every mem kernel form
    (k_mem_lds_lag at config-2 size, k_mem_lds, k_mem), against the oracle."""
    side, total = grid
    ranks = rand_ranks(total, n, seed=1234 + n % 101)
    got = run_plan(t.SWING, t.MEM, side, total, ranks, exec_mode, stride=t.preferred_rank_stride(n),
                   mem_accum=t.ACC_BF16)
    want = [r.copy() for r in ranks]
    oracle.allreduce("mem", t.SWING, side, want, total, acc16=True)
    assert np.array_equal(got, np.stack(want))
    fp32 = [r.copy() for r in ranks]
    oracle.allreduce("mem", t.SWING, side, fp32, total)
    if total >= 8:
        assert not np.array_equal(np.stack(fp32), np.stack(want))   # the two semantics differ


def test_mem_bf16_accumulation_vs_reference_check():
    """How far the reference's own accumulation sits from its ±32 bar on
    config-2 inputs (seed 13, 8x8 mem_2D): recorded in DESIGN.md §2."""
    side, total, n = 8, 64, 327680
    s0, s1, ranks = oracle.reference_inputs(side, total, n, 13)
    got = run_plan(t.SWING, t.MEM, side, total, ranks, t.EXEC_FUSED, mem_accum=t.ACC_BF16)
    bad, maxe = oracle.validate(got[0].view(np.uint32), s0, s1, total, 32.0)
    assert bad > 0 and maxe >= 64     # it does not meet ±32
    got32 = run_plan(t.SWING, t.MEM, side, total, ranks, t.EXEC_FUSED)
    assert oracle.validate(got32[0].view(np.uint32), s0, s1, total, 32.0)[0] == 0
