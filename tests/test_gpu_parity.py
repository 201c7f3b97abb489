"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle.

Integer/byte movement and the per-add bf16 rounding are deterministic, so the
bar is BIT-EXACT equality with the oracle on the same inputs (same schedule,
same add order, each add rounded to nearest even).  The reference's own
tolerance (±32, README.md:31) is checked on top with its validate function.
"""
import numpy as np
import pytest

import oracle
import tenstorrentallreduce_amd as t

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def to_dev(ranks):
    return torch.from_numpy(np.stack(ranks).view(np.int16)).to(DEV)


def from_dev(buf):
    torch.cuda.synchronize()
    return buf.cpu().numpy().view(np.uint16)


def rand_ranks(total, n, seed, lo=0x3F80, hi=0x42C8):
    rng = np.random.default_rng(seed)
    return [rng.integers(lo, hi, n).astype(np.uint16) for _ in range(total)]


def run_plan(algo, variant, side, total, ranks, exec_mode, stride=None):
    n = ranks[0].size
    stride = stride or n
    host = np.zeros((total, stride), dtype=np.uint16)
    for r in range(total):
        host[r, :n] = ranks[r]
    buf = torch.from_numpy(host.view(np.int16)).to(DEV)
    plan = t.Plan(algo, variant, side, n, total, exec_mode)
    ws = torch.empty(max(plan.workspace_bytes, 16), dtype=torch.uint8, device=DEV)
    plan.execute(buf.data_ptr(), stride, ws.data_ptr(), torch.cuda.current_stream())
    out = from_dev(buf)[:, :n]
    plan.close()
    return out


# ------------------------------------------------------------------ bf16 add
def torch_add_ref(a_u16, b_u16):
    a = torch.from_numpy(a_u16.view(np.int16)).view(torch.bfloat16).float()
    b = torch.from_numpy(b_u16.view(np.int16)).view(torch.bfloat16).float()
    return (a + b).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)


@pytest.mark.parametrize("n", [1, 7, 8, 9, 1000, 1 << 20, (1 << 20) + 13])
@pytest.mark.parametrize("offset", [0, 1])
def test_bf16_add_matches_oracle_and_fp32_reference(n, offset):
    rng = np.random.default_rng(n + offset)
    a = rng.integers(0, 0x10000, n + offset).astype(np.uint16)
    b = rng.integers(0, 0x10000, n + offset).astype(np.uint16)
    # keep NaNs out of the bit-exact comparison; covered below
    for x in (a, b):
        nan = (x & 0x7F80) == 0x7F80
        x[nan] &= 0x807F
    da = torch.from_numpy(a.view(np.int16)).to(DEV)
    db = torch.from_numpy(b.view(np.int16)).to(DEV)
    t.bf16_add(da.data_ptr() + 2 * offset, db.data_ptr() + 2 * offset, n, torch.cuda.current_stream())
    got = from_dev(da)[offset:]
    want = np.array([oracle.bf16_add(int(x), int(y)) for x, y in zip(a[offset:offset + 4096], b[offset:offset + 4096])],
                    dtype=np.uint16)
    assert (got[:4096] == want).all()
    ref = torch_add_ref(a[offset:], b[offset:])
    gf = got.astype(np.uint32) << 16
    rf = ref.astype(np.uint32) << 16
    bothnan = np.isnan(gf.view(np.float32)) & np.isnan(rf.view(np.float32))
    assert ((got == ref) | bothnan).all()


def test_bf16_add_nan_inf():
    vals = np.array([0x7F80, 0xFF80, 0x7FC0, 0x0001, 0x8001, 0x7F7F, 0x3F80], dtype=np.uint16)
    a = np.repeat(vals, len(vals))
    b = np.tile(vals, len(vals))
    da = torch.from_numpy(a.view(np.int16)).to(DEV)
    db = torch.from_numpy(b.view(np.int16)).to(DEV)
    t.bf16_add(da.data_ptr(), db.data_ptr(), a.size)
    got = from_dev(da).astype(np.uint32) << 16
    want = torch_add_ref(a, b).astype(np.uint32) << 16
    g, w = got.view(np.float32), want.view(np.float32)
    assert ((g == w) | (np.isnan(g) & np.isnan(w))).all()


def test_bf16_add_masked():
    n_blk, blk = 64, 1024
    rng = np.random.default_rng(3)
    a = rng.integers(0x3F80, 0x42C8, n_blk * blk).astype(np.uint16)
    b = rng.integers(0x3F80, 0x42C8, n_blk * blk).astype(np.uint16)
    mask = 0x9900009999000099
    da = torch.from_numpy(a.view(np.int16)).to(DEV)
    db = torch.from_numpy(b.view(np.int16)).to(DEV)
    t.bf16_add_masked(da.data_ptr(), db.data_ptr(), mask, blk)
    got = from_dev(da)
    summed = torch_add_ref(a, b)
    for k in range(n_blk):
        sl = slice(k * blk, (k + 1) * blk)
        assert (got[sl] == (summed[sl] if (mask >> k) & 1 else a[sl])).all()


# ------------------------------------------------------------------ plans
GRIDS = [(1, 1), (2, 2), (2, 4), (4, 8), (4, 16), (8, 64)]


@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
@pytest.mark.parametrize("variant", ["bo", "lo"])
@pytest.mark.parametrize("algo", [t.SWING_1D, t.RECDUB_1D])
@pytest.mark.parametrize("total", [2, 8, 16, 64])
def test_plan_1d_schedules_bit_exact(total, algo, variant, exec_mode):
    """The prototypes' 1D Swing / RecDub schedules (scratch_work/*_1D) as plans."""
    n = 8 * total * 32
    ranks = rand_ranks(total, n, seed=total + 17 * algo)
    got = run_plan(algo, {"bo": t.BO, "lo": t.LO}[variant], 1, total, ranks, exec_mode)
    want = [r.copy() for r in ranks]
    oracle.allreduce(variant, algo, 1, want, total)
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
@pytest.mark.parametrize("variant", ["bo", "lo", "mem"])
@pytest.mark.parametrize("algo", [t.SWING, t.RECDUB])
@pytest.mark.parametrize("grid", GRIDS)
def test_plan_bit_exact_vs_oracle(grid, algo, variant, exec_mode):
    side, total = grid
    n = 8 * total * 24
    ranks = rand_ranks(total, n, seed=total * 7 + algo)
    got = run_plan(algo, {"bo": t.BO, "lo": t.LO, "mem": t.MEM}[variant], side, total, ranks, exec_mode)
    want = [r.copy() for r in ranks]
    oracle.allreduce(variant, algo, side, want, total)
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("variant", ["bo", "lo", "mem"])
@pytest.mark.parametrize("algo", [t.SWING, t.RECDUB])
@pytest.mark.parametrize("grid", [(2, 4), (4, 16), (8, 64)])
def test_fused_lds_forms_bit_exact(grid, algo, variant):
    """Sizes that take the LDS-staged fused kernels (k_tree_lds, k_butterfly_lds64,
    k_mem_lds: blocks of whole 256-element tiles, >= 256 tiles for LO)."""
    side, total = grid
    n = 256 * total * 8 if total >= 8 else 256 * 64 * 8
    ranks = rand_ranks(total, n, seed=3 * total + algo)
    got = run_plan(algo, {"bo": t.BO, "lo": t.LO, "mem": t.MEM}[variant], side, total, ranks, t.EXEC_FUSED,
                   stride=t.preferred_rank_stride(n))
    want = [r.copy() for r in ranks]
    oracle.allreduce(variant, algo, side, want, total)
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("variant", ["bo", "lo", "mem"])
@pytest.mark.parametrize("algo", [t.SWING, t.RECDUB])
def test_fused_persistent_forms_bit_exact_config2_size(algo, variant):
    """64 ranks x 327,680 bf16 (1280 tiles): the persistent double-buffered
    fused kernels (k_tree_lds_lag, k_butterfly_lds64_pipe,
    k_mem_lds_lag) on random bf16, against the oracle."""
    side, total, n = 8, 64, 327680
    ranks = rand_ranks(total, n, seed=17 + algo)
    got = run_plan(algo, {"bo": t.BO, "lo": t.LO, "mem": t.MEM}[variant], side, total, ranks, t.EXEC_FUSED,
                   stride=t.preferred_rank_stride(n))
    want = [r.copy() for r in ranks]
    oracle.allreduce(variant, algo, side, want, total)
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("variant", ["bo", "lo", "mem"])
def test_fused_chunked_launches_bit_exact(variant):
    """Large buckets run the persistent fused passes as consecutive tile-range
    launches (fused_chunk_tiles, default 1280): 3,904 tiles = three launches
    of 1,301 / 1,301 / 1,302 tiles (ragged), 1.9 MB per rank — against one
    launch over every tile and against the oracle, bit-exact; config 2 stays
    one launch."""
    side, total, n = 8, 64, 3904 * 256
    v = {"bo": t.BO, "lo": t.LO, "mem": t.MEM}[variant]
    ranks = rand_ranks(total, n, seed=41 + v)
    stride = t.preferred_rank_stride(n)
    plan = t.Plan(t.SWING, v, side, n, total, t.EXEC_FUSED)
    assert plan.launches == 3
    with t.tuned(fused_chunk_tiles=0):   # counted with the keys execute reads at launch time
        assert plan.launches == 1
    with t.tuned(fused_form=3):          # a forced single-launch form (the LO register DAG ignores it)
        assert plan.launches == (3 if variant == "lo" else 1)
    plan.close()
    if variant == "lo":   # 1D Swing at 64 ranks has no register DAG: the one-launch butterfly
        plan = t.Plan(t.SWING_1D, v, 1, n, total, t.EXEC_FUSED)
        assert plan.launches == 1
        plan.close()
    plan = t.Plan(t.SWING, v, side, 327680, total, t.EXEC_FUSED)
    assert plan.launches == 1
    plan.close()
    got = run_plan(t.SWING, v, side, total, ranks, t.EXEC_FUSED, stride=stride)
    with t.tuned(fused_chunk_tiles=0):
        one = run_plan(t.SWING, v, side, total, ranks, t.EXEC_FUSED, stride=stride)
    assert (got == one).all()
    want = [r.copy() for r in ranks]
    oracle.allreduce(variant, t.SWING, side, want, total)
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
def test_plan_padded_stride(exec_mode):
    side, total, n = 8, 64, 64 * 8 * 3
    ranks = rand_ranks(total, n, seed=11)
    got = run_plan(t.SWING, t.BO, side, total, ranks, exec_mode, stride=n + 64)
    want = [r.copy() for r in ranks]
    oracle.allreduce("bo", t.SWING, side, want, total)
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
@pytest.mark.parametrize("algo", [t.SWING, t.RECDUB])
def test_config2_reference_inputs(algo, exec_mode):
    """BASELINE config 2: 8x8, 5 tiles per block (640 kB per rank), seed 13."""
    side, total = 8, 64
    n = t.normalize_tiles(5, total, True) * 1024
    s0, s1, ranks = oracle.reference_inputs(side, total, n, 13)
    got = run_plan(algo, t.BO, side, total, ranks, exec_mode)
    want = [r.copy() for r in ranks]
    oracle.allreduce("bo", algo, side, want, total)
    assert (got == np.stack(want)).all()
    for r in (0, 17, 63):
        bad, maxe = oracle.validate(got[r].view(np.uint32), s0, s1, total, 32.0)
        assert bad == 0


@pytest.mark.parametrize("tiles", [1, 2, 16, 64, 128, 320])
@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
def test_lo_sizes_reference_inputs(tiles, exec_mode):
    side, total = 8, 64
    n = t.normalize_tiles(tiles, total, False) * 1024
    s0, s1, ranks = oracle.reference_inputs(side, total, n, 13)
    got = run_plan(t.SWING, t.LO, side, total, ranks, exec_mode)
    want = [r.copy() for r in ranks]
    oracle.allreduce("lo", t.SWING, side, want, total)
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("place,dag", [(1, 1), (0, 1), (1, 0)])
@pytest.mark.parametrize("n", [1024 * 64, 327680])
def test_fused_lo_dag_placement(n, place, dag):
    """The fused Swing 8x8 LO DAG pass through LDS (k_butterfly_lds64_pipe<4>,
    tune lo_dag_reg=0: the register DAG below is the default) with its
    bank-conflict-free node placement (engine.cpp lo_dag_place), with
    first-appearance rows and slots (tune lo_dag_place=0), and the per-rank
    butterfly (lo_dag=0, k_butterfly_lds64_pipe<0>): all bit-exact vs the
    oracle's per-rank butterfly (allred_BO_2D/kernels/dataflow_kernel.cpp:19-29)."""
    side, total = 8, 64
    ranks = rand_ranks(total, n, seed=71 + n % 97)
    with t.tuned(lo_dag_place=place, lo_dag=dag, lo_dag_reg=0):
        got = run_plan(t.SWING, t.LO, side, total, ranks, t.EXEC_FUSED, stride=t.preferred_rank_stride(n))
    want = [r.copy() for r in ranks]
    oracle.allreduce("lo", t.SWING, side, want, total)
    assert (got == np.stack(want)).all()


def signed_ranks(total, n, seed):
    """finite bf16 of both signs from denormals to 2^96 (no overflow in a 64-leaf sum)"""
    rng = np.random.default_rng(seed)
    return [(rng.integers(0, 0x7000, n) | (rng.integers(0, 2, n) << 15)).astype(np.uint16) for _ in range(total)]


@pytest.mark.parametrize("algo,grid", [(t.SWING, (8, 64)), (t.SWING, (8, 32)), (t.SWING_1D, (1, 32))])
@pytest.mark.parametrize("n,pad", [(256, 0), (768, 64), (1024 * 64, 64), (327680, 64), (1 << 20, 0)])
def test_fused_lo_register_dag(algo, grid, n, pad):
    """The fused LO of the non-rank-uniform Swing schedules as the build-time
    DAG of distinct sums evaluated in registers (k_lo_dag_reg, the default from
    lo_dag_reg_min_tiles): one tile, an odd tile count (the persistent grid's
    ragged tail), 128 kB, config-2 size and 2 MiB per rank, padded and unpadded
    rank strides, both signs, denormals to 2^96 — bit-exact vs the oracle's
    per-rank butterfly (allred_LOO_2D/kernels/dataflow_kernel.cpp:127-175)."""
    side, total = grid
    ranks = signed_ranks(total, n, seed=501 + n % 89 + total)
    with t.tuned(lo_dag_reg=1, lo_dag_reg_min_tiles=1):
        got = run_plan(algo, t.LO, side, total, ranks, t.EXEC_FUSED, stride=n + pad)
    want = [r.copy() for r in ranks]
    oracle.allreduce("lo", algo, side, want, total)
    assert (got == np.stack(want)).all()


@pytest.mark.parametrize("lo_tree", [1, 0])
@pytest.mark.parametrize("algo,grid,n", [
    (t.RECDUB, (8, 64), 327680), (t.RECDUB, (8, 64), 1024 * 16), (t.RECDUB, (8, 64), 1024 * 2),
    (t.RECDUB, (4, 16), 1024 * 64),
    (t.RECDUB, (2, 4), 1024), (t.SWING, (4, 16), 1024 * 64), (t.SWING, (2, 4), 1024),
    (t.RECDUB_1D, (8, 64), 1024 * 64), (t.SWING_1D, (2, 4), 1024 * 8)])
def test_fused_lo_rank_uniform_tree_route(algo, grid, n, lo_tree):
    """Schedules whose LO trees are all the same up to child swaps (every RecDub,
    Swing up to 16 ranks) run the fused LO as the BO tree pass (engine.cpp
    lo_rank_uniform); tune lo_tree=0 keeps the butterfly, lo_tree_min_tiles=0
    takes the tree route at every size (by default 64-rank buckets below 64
    tiles keep the butterfly).  Both against the oracle's butterfly, bit-exact."""
    side, total = grid
    ranks = rand_ranks(total, n, seed=29 + total + algo)
    with t.tuned(lo_tree=lo_tree, lo_tree_min_tiles=0 if lo_tree else 64):
        got = run_plan(algo, t.LO, side, total, ranks, t.EXEC_FUSED, stride=t.preferred_rank_stride(n))
    want = [r.copy() for r in ranks]
    oracle.allreduce("lo", algo, side, want, total)
    assert (got == np.stack(want)).all()
    assert (got == got[0]).all()


@pytest.mark.parametrize("n", [1024, 1024 * 8, 1024 * 64])
def test_fused_lo_recdub_default_route(n):
    """64-rank RecDub LO with the default lo_tree_min_tiles (64): the register
    butterfly below 32 kB per rank, the tree pass from there; bit-exact vs the
    oracle either way."""
    ranks = rand_ranks(64, n, seed=41)
    got = run_plan(t.RECDUB, t.LO, 8, 64, ranks, t.EXEC_FUSED, stride=t.preferred_rank_stride(n))
    want = [r.copy() for r in ranks]
    oracle.allreduce("lo", t.RECDUB, 8, want, 64)
    assert (got == np.stack(want)).all()


def test_config1_known_answer():
    s0, s1, ranks = oracle.reference_inputs(2, 4, 1024, -1)
    for exec_mode in (t.EXEC_STEPS, t.EXEC_FUSED):
        got = run_plan(t.RECDUB, t.LO, 2, 4, ranks, exec_mode)
        assert (got == 0x4080).all()  # 4.0


def test_plan_argument_errors():
    with pytest.raises(t.AllredError) as e:
        t.Plan(t.SWING, t.BO, 8, 100, 64)          # not a multiple of 8 * total
    assert e.value.status == -1
    with pytest.raises(t.AllredError) as e:
        t.Plan(t.RECDUB, t.BO, 8, 8 * 16 * 4, 16)   # invalid rectangle
    assert e.value.status == -2
    p = t.Plan(t.SWING, t.LO, 8, 1024, 64)
    with pytest.raises(t.AllredError):
        p.execute(0, 1024)                          # null buffer
    p.close()


# ------------------------------------------------------------------ size-independent properties at full size
@pytest.mark.parametrize("exec_mode", [t.EXEC_STEPS, t.EXEC_FUSED])
def test_config4_sized_bucket_closed_form(exec_mode):
    """1 GiB per rank, 8 ranks (4x2 Swing BO) on one GPU: with the reference
    input convention every later add is an exact doubling, so the result is
    RNE(a+b) * N/2 exactly — checked on the GPU with torch."""
    side, total = 4, 8
    n = (1 << 30) // 2
    g = torch.Generator(device=DEV).manual_seed(5)
    a = (torch.rand(n, generator=g, device=DEV) * 100).to(torch.bfloat16)
    b = (torch.rand(n, generator=g, device=DEV) * 100).to(torch.bfloat16)
    buf = torch.empty((total, n), dtype=torch.bfloat16, device=DEV)
    for r in range(total):
        buf[r] = b if (r % side) % 2 == 0 else a
    plan = t.Plan(t.SWING, t.BO, side, n, total, exec_mode)
    plan.execute(buf.data_ptr(), n, None, torch.cuda.current_stream())
    expect = ((a.float() + b.float()).to(torch.bfloat16).float() * (total // 2)).to(torch.bfloat16)
    for r in range(total):
        assert torch.equal(buf[r], expect), r
    plan.close()


def test_linearity_and_idempotent_layout():
    """allreduce(x) of a rank set that already holds identical vectors v gives
    RNE-doubling chains: N*v exactly for power-of-two N and small v."""
    side, total, n = 8, 64, 64 * 8 * 64
    v = torch.full((n,), 3.0, dtype=torch.bfloat16, device=DEV)
    buf = v.repeat(total, 1).contiguous()
    plan = t.Plan(t.SWING, t.BO, side, n, total, t.EXEC_FUSED)
    plan.execute(buf.data_ptr(), n)
    torch.cuda.synchronize()
    assert torch.equal(buf, torch.full_like(buf, 192.0))
    plan.close()


@pytest.mark.parametrize("grid", [(4, 16), (8, 64)])
@pytest.mark.parametrize("tiles", [1, 5, 40])
def test_fused_bo_on_pinned_host_buckets(grid, tiles):
    """Zero-copy end to end: the fused BO pass on buckets in pinned host memory
    takes the pipelined form (k_tree_lds_pipe: persistent grid, double-buffered
    LDS tiles, looping over more tiles than workgroups at 40 tiles)."""
    side, total = grid
    n = t.normalize_tiles(tiles, total, True) * 1024
    ranks = rand_ranks(total, n, 900 + tiles + total)
    want = [r.copy() for r in ranks]
    oracle.allreduce("bo", t.SWING, side, want, total)
    host = torch.from_numpy(np.stack(ranks).view(np.int16)).pin_memory()
    plan = t.Plan(t.SWING, t.BO, side, n, total, t.EXEC_FUSED)
    plan.execute(host.data_ptr(), n, None, torch.cuda.current_stream())
    torch.cuda.synchronize()
    plan.close()
    assert np.array_equal(host.numpy().view(np.uint16), np.stack(want))
