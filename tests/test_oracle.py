"""The CPU oracle pinned against the reference's fixtures before it is trusted:
the libstdc++ input vectors (tests/golden/inputs_ref.json), the seed -1 known
answer (every element == N) and the reference's own ±32 check."""
import numpy as np
import pytest

import oracle
import tenstorrentallreduce_amd as t


def fnv1a64(words: np.ndarray) -> str:
    h = 1469598103934665603
    for byte in words.astype("<u4").tobytes():
        h ^= byte
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


@pytest.mark.parametrize("impl", ["oracle", "product"])
def test_inputs_match_libstdcxx_generator(golden_inputs, impl):
    gen = oracle.random_bf16_vector if impl == "oracle" else t.random_bf16_vector
    for v in golden_inputs["vectors"]:
        rm = 1 if v["round"] == "rne" else 0
        got = gen(v["bytes"], v["seed"], 100, rm)
        assert [int(x) for x in got[:16]] == v["head"]
        if v["bytes"] <= 2048:
            assert fnv1a64(got) == v["fnv1a64"]
    # full 640 kB hashes, once
    for v in golden_inputs["vectors"]:
        if v["bytes"] == 655360 and v["seed"] in (13, 14):
            got = gen(v["bytes"], v["seed"], 100, 1 if v["round"] == "rne" else 0)
            assert fnv1a64(got) == v["fnv1a64"]


def test_survey_first_values():
    # seed 13 -> 77.5 (trunc) / 78.0 (RNE); seed 14 -> 51.25 / 51.5
    def first(seed, rm):
        w = int(oracle.random_bf16_vector(4, seed, 100, rm)[0]) & 0xFFFF
        return np.array([w << 16], dtype=np.uint32).view(np.float32)[0]
    assert first(13, 0) == 77.5 and first(13, 1) == 78.0
    assert first(14, 0) == 51.25 and first(14, 1) == 51.5


def test_bf16_add_rne():
    # 1 + 2^-8 is a tie between 1 and 1+2^-7 -> even (1.0); 1 + 3*2^-8 -> 1 + 2^-6
    one = 0x3F80
    assert oracle.bf16_add(one, 0x3B80) == one           # + 2^-8
    assert oracle.bf16_add(one, 0x3C40) == 0x3F82        # + 3 * 2^-8
    assert oracle.bf16_add(0x4000, 0xC000) == 0          # 2 - 2


@pytest.mark.parametrize("variant", ["bo", "lo", "mem"])
@pytest.mark.parametrize("side,total", [(2, 4), (8, 64), (4, 8)])
def test_known_answer_all_ones(variant, side, total):
    n = 1024 * total
    s0, s1, ranks = oracle.reference_inputs(side, total, n, -1)
    oracle.allreduce(variant, oracle.SWING, side, ranks, total)
    f = np.array([int(ranks[0][0]) << 16], dtype=np.uint32).view(np.float32)[0]
    assert f == total
    for r in ranks:
        assert (r == ranks[0][0]).all()


@pytest.mark.parametrize("variant", ["bo", "lo", "mem"])
@pytest.mark.parametrize("algo", [oracle.SWING, oracle.RECDUB])
def test_reference_check_passes_at_8x8(variant, algo):
    """Config 2 shape (64 ranks, 5 tiles per block) at seed 13 passes the
    reference's own validate_result_vector with ERROR = 32 on every rank."""
    side, total = 8, 64
    n = (320 if variant != "lo" else 64) * 1024
    s0, s1, ranks = oracle.reference_inputs(side, total, n, 13)
    oracle.allreduce(variant, algo, side, ranks, total)
    for r in range(total):
        bad, _ = oracle.validate(ranks[r].view(np.uint32), s0, s1, total, 32.0)
        assert bad == 0, r


def test_bo_block_equals_lo_tree_of_owner():
    """BO's block b is rank b's LO tree value (reduce-scatter at the owner, then
    all-gather); RecDub LO gives every rank the same value, Swing LO does not."""
    rng = np.random.default_rng(7)
    side, total, blk = 8, 64, 64
    base = [rng.integers(0x3F80, 0x42C8, blk * total).astype(np.uint16) for _ in range(total)]
    for algo in (oracle.SWING, oracle.RECDUB):
        bo = [b.copy() for b in base]
        lo = [b.copy() for b in base]
        oracle.allreduce("bo", algo, side, bo)
        oracle.allreduce("lo", algo, side, lo)
        for r in range(total):
            assert (bo[r] == bo[0]).all()
            assert (bo[0][r * blk:(r + 1) * blk] == lo[r][r * blk:(r + 1) * blk]).all()
        same = all((lo[r] == lo[0]).all() for r in range(total))
        assert same == (algo == oracle.RECDUB)
        if same:  # rank-uniform LO is the BO result (the engine's fused LO route, engine.cpp lo_rank_uniform)
            assert all((lo[r] == bo[r]).all() for r in range(total))


def test_loopback_config1_known_answer():
    out = oracle.loopback("bo", [0, 1, 2, -1, 1, 32, 0, 0], reps=3)
    assert out["mismatches"] == 0 and out["ranks"] == 4 and out["bytes_per_rank"] == 2048
    assert "All values match!" in out["stdout"]


@pytest.mark.parametrize("variant,argv", [
    ("bo", [1, 1, 8, 13, 1, 32, 0, 1]),   # 8x8 Swing BO, 128 kB
    ("bo", [0, 1, 8, 13, 1, 32, 5, 1]),   # 8x8 RecDub BO, print core 5
    ("bo", [1, 1, 8, 13, 16, 32, 0, 0]),  # 8x8 Swing LO 32 kB (LOO path)
    ("mem", [1, 1, 8, 13, 1, 32]),
])
def test_loopback_multiprocess(variant, argv):
    out = oracle.loopback(variant, argv, reps=2)
    assert out["mismatches"] == 0 and out["ranks"] == 64


def test_loopback_profile_log_per_rank_stats(tmp_path):
    """Per-rank ALL_RED_LOOP stamps in the profile_log_device.csv layout, read
    back with the reference analyzer's statistics (tools/profile_analyzer.py)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from profile_analyzer import analyze
    log = str(tmp_path / "profile_log_device.csv")
    out = oracle.loopback("bo", [1, 1, 4, 13, 1, 32, 0, 1], reps=3, total=8, profile_log=log)
    assert out["mismatches"] == 0
    lines = open(log).read().splitlines()
    assert lines[0].startswith("ARCH:") and len(lines) == 2 + 3 * 8 * 2
    r = analyze(log)
    assert r["cores"] == 8
    assert 0 < r["min"] <= r["q1"] <= r["median"] <= r["q3"] <= r["max"]
    # the last rep's per-rank span never exceeds that rep's max-end - min-start
    assert r["max"] <= out["seconds"][-1] * 1e9 + 1
