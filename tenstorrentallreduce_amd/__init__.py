"""MI355X-native allreduce engine with the capabilities of
EngineerCharlie/TenstorrentAllreduce (2D Swing / Recursive-Doubling
allreduce, bandwidth-optimal / latency-optimal / shared-memory variants).

The engine is C++/HIP (``liballred.so``, C-ABI in ``include/allred.h``) plus
the reference's executables (``bin/allred_BO_2D`` ...).  This package is a
thin Python view of that C-ABI for tests and ``bench.py``: device memory and
streams come from PyTorch (plumbing), every computation runs in the library.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Callable, Sequence

import numpy as np

from . import _lib
from ._lib import (ACC_BF16, ACC_FP32, BO, EXEC_FUSED, EXEC_STEPS, LO, MEM, MULTI_FLAT, MULTI_HIER,  # noqa: F401
                   MULTI_LOCAL, RECDUB, RECDUB_1D, SWING, SWING_1D, TRANSPORT_HOST, TRANSPORT_PEER, TRANSPORT_RCCL,
                   AllredError, Args, DistDesc, MultiOpts, MultiPlan, PlanDesc, Report, Schedule, Seg, check, lib)

__all__ = [
    "BO", "LO", "MEM", "SWING", "RECDUB", "SWING_1D", "RECDUB_1D", "get_comm_partner_swing_1D",
    "get_comm_partner_recdub_1D", "EXEC_STEPS", "EXEC_FUSED", "AllredError", "schedule",
    "highest_power_of_two", "get_step_directions", "get_comm_partner_swing_2D", "get_comm_partner_recdub_2D",
    "get_swing_block_comm_indexes", "get_recdub_block_comm_indexes", "normalize_tiles",
    "random_bf16_vector", "constant_bf16_vector", "validate_result_vector", "Plan", "preferred_rank_stride", "bf16_add",
    "bf16_add_masked", "tree_reduce", "broadcast", "parse_args", "run", "run_cli", "Comm", "dist_desc", "dist_allreduce",
    "dist_allreduce_host", "dist_allreduce_pipelined", "tree_broadcast_pipelined", "dist_workspace_bytes", "dist_program_stats", "Peer", "tune", "tuned", "last_launch",
    "ACC_FP32",
    "ACC_BF16", "multi_plan", "run_multi", "TRANSPORT_RCCL", "TRANSPORT_PEER", "TRANSPORT_HOST", "MULTI_FLAT",
    "MULTI_HIER", "MULTI_LOCAL",
]


# ---------------------------------------------------------------- tuning
def tune(key: str, value: int | None = None) -> int:
    """allred_tune_set / allred_tune_get: switch between bit-identical kernel
    forms (A/B); returns the previous value.  Keys: allred.h §Tuning."""
    old = C.c_int64(0)
    check(lib.allred_tune_get(key.encode(), C.byref(old)), f"tune_get({key})")
    if value is not None:
        check(lib.allred_tune_set(key.encode(), int(value)), f"tune_set({key}={value})")
    return old.value


class tuned:
    """with tuned(key=value, ...): the keys set for the block, restored after."""

    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = tune(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            tune(k, v)


def last_launch() -> dict:
    """allred_last_launch: the kernel this thread's last reported launch ran, the
    grid its launcher chose, its static LDS / VGPRs, the workgroups per CU that can
    be resident and the device's CU count."""
    li = _lib.LaunchInfo()
    check(lib.allred_last_launch(C.byref(li)), "last_launch")
    return {"kernel": li.kernel.decode(), "grid": li.grid, "block": li.block, "lds_bytes": li.lds_bytes,
            "vgprs": li.regs, "resident_per_cu": li.resident_per_cu, "cus": li.cus,
            "grid_resident": li.grid <= li.resident_per_cu * li.cus}


# ---------------------------------------------------------------- schedule
def highest_power_of_two(v: int) -> int:  # allred_helper.cpp:122
    return lib.allred_highest_power_of_two(v)


def get_step_directions(x: int, y: int) -> int:  # allred_helper.cpp:136
    return lib.allred_get_step_directions(x, y)


def get_comm_partner_swing_2D(node, step, horizontal_step, side, total) -> int:  # allred_helper.cpp:166
    return lib.allred_get_comm_partner_swing_2d(node, step, int(bool(horizontal_step)), side, total)


def get_comm_partner_recdub_2D(node, step, horizontal_step, depth, step_directions, side):
    """allred_helper.cpp:145; returns (partner, updated step_directions)."""
    d = C.c_uint32(step_directions)
    p = lib.allred_get_comm_partner_recdub_2d(node, step, int(bool(horizontal_step)), depth, C.byref(d), side)
    return p, d.value


def get_swing_block_comm_indexes(node, step, blocks, horizontal_step, side, total) -> int:
    """allred_BO_2D.cpp:220; ORs into the 64-bit mask `blocks`, returns it."""
    b = (C.c_uint32 * 2)(blocks & 0xFFFFFFFF, blocks >> 32)
    lib.allred_get_swing_block_comm_indexes(node, step, b, int(bool(horizontal_step)), side, total)
    return b[0] | (b[1] << 32)


def get_recdub_block_comm_indexes(node, step, blocks, horizontal_step, side, total, depth, step_directions=0):
    """allred_BO_2D.cpp:242; returns (mask, step_directions)."""
    b = (C.c_uint32 * 2)(blocks & 0xFFFFFFFF, blocks >> 32)
    d = C.c_uint32(step_directions)
    lib.allred_get_recdub_block_comm_indexes(node, step, b, int(bool(horizontal_step)), side, total, depth,
                                             C.byref(d))
    return b[0] | (b[1] << 32), d.value


def get_comm_partner_swing_1D(node: int, step: int, num_nodes: int) -> int:  # all_red_swing_1D.cpp:32
    return lib.allred_get_comm_partner_swing_1d(node, step, num_nodes)


def get_comm_partner_recdub_1D(node: int, step: int, step_directions: int = 0):  # recdub_multicore_1D.cpp:165
    d = C.c_uint32(step_directions)
    p = lib.allred_get_comm_partner_recdub_1d(node, step, C.byref(d))
    return p, d.value


def normalize_tiles(tiles: int, total_nodes: int, large_buffer: bool) -> int:  # allred_helper.cpp:224
    return lib.allred_normalize_tiles(tiles, total_nodes, int(bool(large_buffer)))


def schedule(algo: int, side: int, total: int | None = None) -> dict:
    """The per-rank schedule of allred_BO_2D.cpp:75-212 (validated)."""
    total = side * side if total is None else total
    s = Schedule()
    check(lib.allred_schedule_build(algo, side, total, C.byref(s)), f"schedule({algo},{side},{total})")
    T, K = s.total, s.steps
    return {
        "algo": s.algo, "side": s.side, "total": T, "steps": K,
        "partner": [[s.partner[r][k] for k in range(K)] for r in range(T)],
        "send": [[s.send[r][k] for k in range(K)] for r in range(T)],
        "recv": [[s.recv[r][k] for k in range(K)] for r in range(T)],
        "dirs": [s.dirs[r] for r in range(T)],
        "tree_order": [[s.tree_order[x][i] for i in range(T)] for x in range(T)],
    }


# ---------------------------------------------------------------- host data
def random_bf16_vector(num_bytes: int, seed: int, rand_max: int = 100, round_mode: int = 0) -> np.ndarray:
    """tt-metal create_random_vector_of_bfloat16 (packed uint32, low half first)."""
    out = np.empty(num_bytes // 4, dtype=np.uint32)
    lib.allred_random_bf16_vector(num_bytes, rand_max, seed, round_mode, out.ctypes.data)
    return out


def constant_bf16_vector(num_bytes: int, value: float) -> np.ndarray:
    out = np.empty(num_bytes // 4, dtype=np.uint32)
    lib.allred_constant_bf16_vector(num_bytes, value, out.ctypes.data)
    return out


def validate_result_vector(result, src0, src1, num_els: int, error: float, total_nodes: int,
                           verbose: bool = False):
    """allred_helper.cpp:18-120; returns (mismatches, max_error)."""
    arrs = [np.ascontiguousarray(x, dtype=np.uint32) for x in (result, src0, src1)]
    m = C.c_float(0)
    bad = lib.allred_validate_result_vector(arrs[0].ctypes.data, arrs[1].ctypes.data, arrs[2].ctypes.data,
                                            num_els, error, total_nodes, int(verbose), C.byref(m))
    return int(bad), float(m.value)


# ---------------------------------------------------------------- device
def _stream_ptr(stream) -> int | None:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


def bf16_add(dst_ptr: int, src_ptr: int, n: int, stream=None) -> None:
    check(lib.allred_bf16_add(dst_ptr, src_ptr, n, _stream_ptr(stream)), "bf16_add")


def bf16_add_masked(dst_ptr: int, src_ptr: int, mask: int, block_elems: int, stream=None) -> None:
    check(lib.allred_bf16_add_masked(dst_ptr, src_ptr, mask, block_elems, _stream_ptr(stream)), "bf16_add_masked")


def tree_reduce(ranks_ptr: int, stride: int, n: int, algo: int, side: int, total: int, out_ptr: int,
                stream=None) -> None:
    check(lib.allred_tree_reduce(ranks_ptr, stride, n, algo, side, total, out_ptr, _stream_ptr(stream)),
          "tree_reduce")


def broadcast(ranks_ptr: int, stride: int, n: int, total: int, src_ptr: int, stream=None) -> None:
    check(lib.allred_broadcast(ranks_ptr, stride, n, total, src_ptr, _stream_ptr(stream)), "broadcast")


def preferred_rank_stride(elems: int) -> int:
    return lib.allred_preferred_rank_stride(elems)


class Plan:
    """N virtual ranks in one GPU's HBM (allred_plan_*).  exec_mode: EXEC_FUSED
    (default, one HBM pass) or EXEC_STEPS (the reference's step structure);
    mem_accum (MEM): ACC_FP32 or ACC_BF16 (the reference's bf16 dest)."""

    def __init__(self, algo: int, variant: int, side: int, elems_per_rank: int, total: int = 0,
                 exec_mode: int = EXEC_FUSED, device: int = -1, mem_accum: int = ACC_FP32):
        d = PlanDesc(algo, variant, exec_mode, side, total, device, elems_per_rank, mem_accum)
        h = C.c_void_p()
        check(lib.allred_plan_create(C.byref(d), C.byref(h)), "plan_create")
        self._h = h
        self.total = total or side * side
        self.elems = elems_per_rank
        self.workspace_bytes = lib.allred_plan_workspace_bytes(h)
        self.stamp_words = lib.allred_plan_stamp_words(h)

    @property
    def launches(self) -> int:
        """Kernel launches one execute enqueues now (fused plans: with the current tune keys)."""
        return lib.allred_plan_launches(self._h)

    def execute(self, ranks_ptr: int, stride: int, workspace_ptr: int | None = None, stream=None,
                stamps_ptr: int | None = None) -> None:
        """stamps_ptr: device memory of stamp_words uint64 (schedule form only)."""
        check(lib.allred_plan_execute_profiled(self._h, ranks_ptr, stride, workspace_ptr, stamps_ptr,
                                               _stream_ptr(stream)), "plan_execute")

    def rank_zones(self, stamps: np.ndarray):
        """Per-rank ALL_RED_LOOP (start, end) in 100 MHz ticks from host stamps."""
        st = np.ascontiguousarray(stamps, dtype=np.uint64)
        zs = np.zeros(self.total, dtype=np.uint64)
        ze = np.zeros(self.total, dtype=np.uint64)
        check(lib.allred_plan_rank_zones(self._h, st.ctypes.data, zs.ctypes.data, ze.ctypes.data), "plan_rank_zones")
        return zs, ze

    def close(self):
        if self._h:
            lib.allred_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- program surface
def parse_args(argv: Sequence[str], variant: int = BO) -> Args:
    arr = (C.c_char_p * len(argv))(*[a.encode() for a in argv])
    a = Args()
    check(lib.allred_args_parse(len(argv), arr, variant, C.byref(a)), "args_parse")
    return a


def run(argv: Sequence[str], variant: int = BO, verbose: bool = False, exec_mode: int | None = None) -> Report:
    """AllredConfig(argv) + RunProgram() in-process (allred_helper.hpp:47-97)."""
    a = parse_args(argv, variant)
    if exec_mode is not None:
        a.exec = exec_mode
    r = Report()
    check(lib.allred_run(C.byref(a), int(verbose), C.byref(r)), "run")
    return r


def run_cli(binary: str, args: Sequence[str], env: dict | None = None, timeout: float = 300):
    """Run bin/<binary> (allred_BO_2D / allred_LO_2D / allred_mem_2D) like the reference."""
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([os.path.join(_lib.BIN_DIR, binary), *map(str, args)], capture_output=True, text=True,
                          env=e, timeout=timeout)


def multi_plan(argv: Sequence[str], variant: int = BO, gpus: int | None = None, check_all: bool = False) -> MultiPlan:
    """The plan of allred_run across GPUs (allred_multi_plan_build): pure host
    computation, no HIP call.  gpus overrides argv[10] / ALLRED_GPUS."""
    a = parse_args(argv, variant)
    if gpus is not None:
        a.gpus = gpus
    p = MultiPlan()
    check(lib.allred_multi_plan_build(C.byref(a), int(check_all), C.byref(p)), "multi_plan_build")
    return p


def run_multi(argv: Sequence[str], variant: int = BO, gpus: int | None = None, transport: int = TRANSPORT_RCCL,
              share_device: bool = False, timeout_ms: int = 0, verbose: bool = False, outputs: bool = True,
              inputs: np.ndarray | None = None):
    """allred_run across GPUs with an explicit backend (allred_run_multi).
    inputs: None (the reference's generated, validated inputs) or a (total,
    elems) uint16 array of arbitrary rank vectors (validation skipped).
    Returns (Report, every rank's result as a (total, elems) uint16 array or None)."""
    a = parse_args(argv, variant)
    if gpus is not None:
        a.gpus = gpus
    n = a.num_tiles * 1024
    r = Report()
    out = np.zeros((a.total_nodes, n), dtype=np.uint16) if outputs else None
    inp = None
    if inputs is not None:
        inp = np.ascontiguousarray(inputs, dtype=np.uint16)
        if inp.shape != (a.total_nodes, n):
            raise ValueError(f"inputs must be ({a.total_nodes}, {n})")
    o = MultiOpts(transport, int(share_device), timeout_ms, 0)
    check(lib.allred_run_multi(C.byref(a), C.byref(o), int(verbose), C.byref(r),
                               None if inp is None else inp.ctypes.data, None if out is None else out.ctypes.data),
          "run_multi")
    return r, out


# ---------------------------------------------------------------- multi-GPU
class Comm:
    """One RCCL communicator per process/GPU (allred_comm_*)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * _lib.UNIQUE_ID_BYTES)()
        check(lib.allred_comm_get_unique_id(buf), "comm_get_unique_id")
        return bytes(buf)

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int):
        buf = (C.c_uint8 * _lib.UNIQUE_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib.allred_comm_init(buf, nranks, rank, device, C.byref(h)), "comm_init")
        self._h = h
        self.nranks, self.rank = nranks, rank

    @classmethod
    def init_all(cls, devices: Sequence[int]) -> list:
        """One communicator per device in this process (allred_comm_init_all)."""
        devs = (C.c_int * len(devices))(*devices)
        hs = (C.c_void_p * len(devices))()
        check(lib.allred_comm_init_all(len(devices), devs, hs), "comm_init_all")
        out = []
        for i, h in enumerate(hs):
            c = cls.__new__(cls)
            c._h = C.c_void_p(h)
            c.nranks, c.rank = len(devices), i
            out.append(c)
        return out

    def set_timeout(self, ms: int) -> None:
        check(lib.allred_comm_set_timeout(self._h, ms), "comm_set_timeout")

    def wait(self, stream=None) -> None:
        """Bounded stream drain (allred_comm_wait): ALLRED_ERR_TRANSPORT past the deadline."""
        check(lib.allred_comm_wait(self._h, _stream_ptr(stream)), "comm_wait")

    @property
    def aborted(self) -> bool:
        return bool(lib.allred_comm_aborted(self._h))

    def close(self):
        if self._h:
            lib.allred_comm_destroy(self._h)
            self._h = None


def dist_desc(algo: int, variant: int, side: int, total: int, elems: int, local_ranks: int = 1,
              local_side: int = 1, local_algo: int = SWING, channels: int = 0, mem_accum: int = ACC_FP32) -> DistDesc:
    return DistDesc(algo, variant, side, total, elems, local_ranks, local_side, local_algo, channels, mem_accum)


def dist_workspace_bytes(desc: DistDesc) -> int:
    return lib.allred_dist_workspace_bytes(C.byref(desc))


def dist_program_stats(desc: DistDesc, rank: int) -> dict:
    """The cached per-rank program: exchange steps, add launches, send+recv segments."""
    k, a, g = C.c_int(0), C.c_int(0), C.c_int(0)
    check(lib.allred_dist_program_stats(C.byref(desc), rank, C.byref(k), C.byref(a), C.byref(g)), "dist_program_stats")
    return {"steps": k.value, "add_launches": a.value, "segments": g.value}


def dist_allreduce(comm: Comm, desc: DistDesc, buf_ptr: int, workspace_ptr: int, stream=None) -> None:
    check(lib.allred_dist_allreduce(comm._h, C.byref(desc), buf_ptr, workspace_ptr, _stream_ptr(stream)),
          "dist_allreduce")


def dist_allreduce_pipelined(comm: Comm, desc: DistDesc, cur_ptr: int | None, workspace_ptr: int, stream=None) -> None:
    """The hierarchical step pipelined across buckets (allred_dist_allreduce_pipelined):
    K buckets = K + 1 calls b0, b1, ..., None; workspace = 2 * dist_workspace_bytes(desc)."""
    check(lib.allred_dist_allreduce_pipelined(comm._h, C.byref(desc), cur_ptr or None, workspace_ptr,
                                              _stream_ptr(stream)), "dist_allreduce_pipelined")


def tree_broadcast_pipelined(cur_ptr: int, prev_ptr: int, stride: int, n: int, algo: int, side: int, total: int,
                             cur_out_ptr: int, prev_src_ptr: int, stream=None) -> None:
    check(lib.allred_tree_broadcast_pipelined(cur_ptr, prev_ptr, stride, n, algo, side, total, cur_out_ptr,
                                              prev_src_ptr, _stream_ptr(stream)), "tree_broadcast_pipelined")


def dist_allreduce_host(desc: DistDesc, rank: int, buf: np.ndarray, scratch: np.ndarray,
                        exchange: Callable[[int, list, list], None]) -> None:
    """Host-memory twin: `exchange(peer, sends, recvs)` gets lists of writable
    uint8 numpy views and must send every send view / fill every recv view."""

    def _cb(_ctx, peer, nsend, send, nrecv, recv):
        try:
            def views(segs, n):
                out = []
                for i in range(n):
                    s = segs[i]
                    out.append(np.ctypeslib.as_array((C.c_uint8 * s.bytes).from_address(s.ptr)))
                return out
            exchange(peer, views(send, nsend), views(recv, nrecv))
            return 0
        except Exception:  # pragma: no cover - surfaced as ALLRED_ERR_TRANSPORT
            import traceback
            traceback.print_exc()
            return 1

    cb = _lib.EXCHANGE_FN(_cb)
    assert buf.dtype == np.uint16 and scratch.dtype == np.uint16
    check(lib.allred_dist_allreduce_host(C.byref(desc), rank, buf.ctypes.data, scratch.ctypes.data, cb, None),
          "dist_allreduce_host")


PEER_TIMEOUT, PEER_WIN_CACHED, PEER_FLAGS_CACHED = _lib.PEER_TIMEOUT, _lib.PEER_WIN_CACHED, _lib.PEER_FLAGS_CACHED


class Peer:
    """Peer-mapped one-shot allreduce across GPUs (allred_peer_*): the
    allred_mem_2D variant over xGMI.  handle() -> exchange with every rank ->
    connect(list of all ranks' handles in rank order)."""

    def __init__(self, nranks: int, rank: int, device: int, max_elems: int):
        h = C.c_void_p()
        check(lib.allred_peer_create(nranks, rank, device, max_elems, C.byref(h)), "peer_create")
        self._h = h
        self.nranks, self.rank = nranks, rank

    def handle(self) -> bytes:
        buf = (C.c_uint8 * _lib.PEER_HANDLE_BYTES)()
        check(lib.allred_peer_handle(self._h, buf), "peer_handle")
        return bytes(buf)

    def connect(self, handles: Sequence[bytes]) -> None:
        blob = b"".join(handles)
        arr = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        check(lib.allred_peer_connect(self._h, arr), "peer_connect")

    @staticmethod
    def connect_all(peers: Sequence["Peer"]) -> None:
        """The peers of ONE process (peers[q] = rank q), mapped into each other
        without IPC (allred_peer_connect_all)."""
        arr = (C.c_void_p * len(peers))(*[p._h.value for p in peers])
        check(lib.allred_peer_connect_all(len(peers), arr), "peer_connect_all")

    def allreduce(self, buf_ptr: int, elems: int, stream=None, local_ranks: int = 1, local_side: int = 1,
                  local_algo: int = SWING, workspace_ptr: int | None = None, check_status: bool = False) -> None:
        """check_status: synchronise the stream and raise AllredError(ERR_TRANSPORT)
        if a peer wait timed out (the bytes are then wrong).  Without it the
        caller must call check() (or status()) before using the result."""
        check(lib.allred_peer_allreduce(self._h, buf_ptr, elems, local_ranks, local_side, local_algo, workspace_ptr,
                                        _stream_ptr(stream)), "peer_allreduce")
        if check_status:
            self.check(stream)

    def allreduce_pipelined2(self, cur_ptr: int | None, elems: int, stream=None, local_ranks: int = 64,
                             local_side: int = 8, local_algo: int = SWING) -> None:
        """The hierarchical step pipelined two buckets deep (k_hier_x2): starts cur,
        sums the owned tiles of the previous call's bucket, writes the rows of the
        bucket started two calls earlier; cur None finishes everything pending.
        K buckets = K + 1 calls: b0, b1, ..., b_{K-1}, None."""
        check(lib.allred_peer_allreduce_pipelined2(self._h, cur_ptr or None, elems, local_ranks, local_side,
                                                   local_algo, _stream_ptr(stream)), "peer_allreduce_pipelined2")

    def dist_allreduce(self, desc: DistDesc, buf_ptr: int, workspace_ptr: int | None = None, stream=None,
                       check_status: bool = False) -> None:
        """dist_allreduce's program (same desc, same bits) over the peer windows."""
        check(lib.allred_peer_dist_allreduce(self._h, C.byref(desc), buf_ptr, workspace_ptr, _stream_ptr(stream)),
              "peer_dist_allreduce")
        if check_status:
            self.check(stream)

    def check(self, stream=None) -> None:
        """allred_peer_check: sync `stream`, raise if any call so far timed out."""
        check(lib.allred_peer_check(self._h, _stream_ptr(stream)), "peer timeout (a peer never arrived)")

    def set_oneshot_max(self, nbytes: int) -> None:
        """Buckets of at most nbytes run as one kernel (same bits either way)."""
        check(lib.allred_peer_set_oneshot_max(self._h, nbytes), "peer_set_oneshot_max")

    def set_hier_ll(self, mode) -> None:
        """64 local ranks: 1 (or True, the default) the hierarchical step as one
        launch with LL push hand-offs, reducing and writing waves in every
        workgroup (k_hier_ws); 0 (or False) the launch form.  Same result bits."""
        check(lib.allred_peer_set_hier_ll(self._h, int(mode)), "peer_set_hier_ll")

    def set_lo_ll_max(self, nbytes: int) -> None:
        """One-channel LO buckets up to nbytes take the LL-push program (same bits; 0 = never)."""
        check(lib.allred_peer_set_lo_ll_max(self._h, nbytes), "peer_set_lo_ll_max")

    def set_mem_ll_max(self, nbytes: int) -> None:
        """mem_2D buckets up to nbytes take the LL-push form (same bits; 0 = never)."""
        check(lib.allred_peer_set_mem_ll_max(self._h, nbytes), "peer_set_mem_ll_max")

    def set_sched_push(self, min_bytes: int) -> None:
        """BO buckets of >= min_bytes in the push form of the scheduled program (0 = never)."""
        check(lib.allred_peer_set_sched_push(self._h, min_bytes), "peer_set_sched_push")

    def set_max_groups(self, groups: int) -> None:
        """Grid cap of the hierarchical one-kernel forms (0 = one full grid per GPU);
        processes sharing a GPU need groups <= 512 / processes."""
        check(lib.allred_peer_set_max_groups(self._h, groups), "peer_set_max_groups")

    def status(self) -> int:
        v = C.c_uint32(0)
        check(lib.allred_peer_status(self._h, C.byref(v)), "peer_status")
        return v.value

    def clear_status(self) -> None:
        """allred_peer_clear_status: the sticky timeout bit cleared (no kernel of this peer in flight)"""
        check(lib.allred_peer_clear_status(self._h), "peer_clear_status")

    def close(self):
        if self._h:
            lib.allred_peer_destroy(self._h)
            self._h = None
