"""CPU ORACLE — Python view of oracle/build/liballred_oracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline, never by the
product (tenstorrentallreduce_amd/).  See allred_oracle.h for what is
restated from where and how parity is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "liballred_oracle.so")
CLI = os.path.join(HERE, "build", "allred_oracle_cli")


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


if not os.path.exists(SO):
    build()

_o = C.CDLL(SO)


class Schedule(C.Structure):
    _fields_ = [("swing", C.c_int), ("side", C.c_int), ("total", C.c_int), ("steps", C.c_int),
                ("partner", (C.c_int * 6) * 64), ("send", (C.c_uint64 * 6) * 64),
                ("recv", (C.c_uint64 * 6) * 64), ("dirs", C.c_uint32 * 64)]


_o.or_bf16_rne.restype = C.c_uint16
_o.or_bf16_rne.argtypes = [C.c_float]
_o.or_bf16_trunc.restype = C.c_uint16
_o.or_bf16_trunc.argtypes = [C.c_float]
_o.or_bf16_add.restype = C.c_uint16
_o.or_bf16_add.argtypes = [C.c_uint16, C.c_uint16]
_o.or_random_bf16_vector.argtypes = [C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_void_p]
_o.or_constant_bf16_vector.argtypes = [C.c_size_t, C.c_float, C.c_void_p]
_o.or_build_schedule.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(Schedule)]
_o.or_normalize_tiles.argtypes = [C.c_int, C.c_int, C.c_int]
_o.or_highest_power_of_two.argtypes = [C.c_int]
_o.or_step_directions.restype = C.c_uint32
_o.or_step_directions.argtypes = [C.c_int, C.c_int]
for f in ("or_allreduce_bo", "or_allreduce_lo"):
    getattr(_o, f).argtypes = [C.POINTER(Schedule), C.POINTER(C.c_void_p), C.c_size_t]
_o.or_allreduce_mem.argtypes = [C.c_int, C.POINTER(C.c_void_p), C.c_size_t]
_o.or_allreduce_mem_acc.argtypes = [C.c_int, C.POINTER(C.c_void_p), C.c_size_t, C.c_int]
_o.or_validate.restype = C.c_long
_o.or_validate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_float, C.c_uint32, C.c_int,
                           C.POINTER(C.c_float)]

SWING, RECDUB, RECDUB_1D, SWING_1D = 1, 0, 2, 3


def bf16_add(a: int, b: int) -> int:
    return _o.or_bf16_add(a, b)


def random_bf16_vector(num_bytes: int, seed: int, rand_max: int = 100, round_mode: int = 0) -> np.ndarray:
    out = np.empty(num_bytes // 4, dtype=np.uint32)
    _o.or_random_bf16_vector(num_bytes, rand_max, seed, round_mode, out.ctypes.data)
    return out


def constant_bf16_vector(num_bytes: int, value: float) -> np.ndarray:
    out = np.empty(num_bytes // 4, dtype=np.uint32)
    _o.or_constant_bf16_vector(num_bytes, value, out.ctypes.data)
    return out


def highest_power_of_two(v: int) -> int:
    return _o.or_highest_power_of_two(v)


def step_directions(x: int, y: int) -> int:
    return _o.or_step_directions(x, y)


def normalize_tiles(tiles: int, total: int, large: bool) -> int:
    return _o.or_normalize_tiles(tiles, total, int(large))


def schedule(swing: int, side: int, total: int | None = None):
    total = side * side if total is None else total
    s = Schedule()
    st = _o.or_build_schedule(swing, side, total, C.byref(s))
    return st, s


def _ptrs(ranks):
    return (C.c_void_p * len(ranks))(*[r.ctypes.data for r in ranks])


def allreduce(variant: str, swing: int, side: int, ranks: list[np.ndarray], total: int | None = None,
              acc16: bool = False) -> None:
    """In-place allreduce of uint16 bf16 rank vectors: variant bo | lo | mem
    (acc16: mem with the reference's bf16 accumulation, every add rounded)."""
    total = len(ranks) if total is None else total
    n = ranks[0].size
    if variant == "mem":
        st = _o.or_allreduce_mem_acc(total, _ptrs(ranks), n, int(acc16))
    else:
        rc, s = schedule(swing, side, total)
        assert rc == 0, "invalid grid"
        st = getattr(_o, f"or_allreduce_{variant}")(C.byref(s), _ptrs(ranks), n)
    assert st == 0


def validate(result, src0, src1, total_nodes: int, error: float, trgt_mode: int = 0):
    m = C.c_float(0)
    r = np.ascontiguousarray(result, dtype=np.uint32)
    a = np.ascontiguousarray(src0, dtype=np.uint32)
    b = np.ascontiguousarray(src1, dtype=np.uint32)
    bad = _o.or_validate(r.ctypes.data, a.ctypes.data, b.ctypes.data, a.size, error, total_nodes, trgt_mode,
                         C.byref(m))
    return int(bad), float(m.value)


def reference_inputs(side: int, total: int, n_elems: int, seed: int, round_mode: int = 0):
    """Rank vectors of the reference convention (allred_helper.cpp:277-285,
    allred_BO_2D.cpp:79-85): even x gets src_1 (seed+1), odd x gets src_0."""
    nbytes = n_elems * 2
    if seed < 0:
        s0 = constant_bf16_vector(nbytes, 1.0)
        s1 = s0.copy()
    else:
        s0 = random_bf16_vector(nbytes, seed, 100, round_mode)
        s1 = random_bf16_vector(nbytes, seed + 1, 100, round_mode)
    ranks = [(s1 if (r % side) % 2 == 0 else s0).view(np.uint16).copy() for r in range(total)]
    return s0, s1, ranks


def loopback(variant: str, argv: list, reps: int = 5, total: int = 0, round_mode: int = 0, timeout: float = 600,
             profile_log: str | None = None):
    """Run the multi-process loopback restatement; returns its JSON summary.
    profile_log: also write per-rank ALL_RED_LOOP stamps there (tt-metal
    profile_log_device.csv layout)."""
    import json
    args = [CLI, variant, *map(str, argv)]
    while len(args) < 10:
        args.append("0")
    args += [str(reps), str(total), str(round_mode)]
    env = dict(os.environ)
    if profile_log:
        env["ORACLE_PROFILE_LOG"] = profile_log
    p = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env)
    if p.returncode != 0:
        raise RuntimeError(p.stderr)
    first = p.stdout.splitlines()[0]
    out = json.loads(first)
    out["stdout"] = p.stdout
    return out
