"""ctypes binding of liballred.so (include/allred.h).

The product is the C-ABI library built in-tree by ``make -C
tenstorrentallreduce_amd`` (``__graft_entry__.build()``).  This module only
declares its symbols; there is no Python or CPU fallback for any device entry
point — if the library is missing, importing the package fails loudly.

HIP runtime note: ``import torch`` must come before the library is loaded so
that liballred.so binds (by soname ``libamdhip64.so.7`` / ``librccl.so.1``)
to the one HIP runtime and RCCL torch already loaded, never a second copy.
"""
from __future__ import annotations

import ctypes as C
import os

try:  # plumbing only: one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# ALLRED_LIB_PATH: another build of the same ABI (A/B timing of a change, tools/gpu_mem_ab.sh)
LIB_PATH = os.environ.get("ALLRED_LIB_PATH") or os.path.join(HERE, "lib", "liballred.so")
BIN_DIR = os.path.join(HERE, "bin")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build the HIP engine first "
        "(python -c 'import __graft_entry__ as g; g.build()' or make -C tenstorrentallreduce_amd)")

lib = C.CDLL(LIB_PATH)

# ---- status / enums (allred.h) ------------------------------------------
OK, ERR_ARG, ERR_SCHEDULE, ERR_HIP, ERR_RCCL, ERR_NOMEM, ERR_UNSUPPORTED, ERR_TRANSPORT = 0, -1, -2, -3, -4, -5, -6, -7
RECDUB, SWING, RECDUB_1D, SWING_1D = 0, 1, 2, 3
BO, LO, MEM = 0, 1, 2
STEPS_REG = 0x100   # allred_steps_program: | ALLRED_BO -> the register-staged form's program
EXEC_STEPS, EXEC_FUSED = 0, 1
ACC_FP32, ACC_BF16 = 0, 1
ABI_VERSION = 7
MAX_NODES, MAX_STEPS = 64, 6
UNIQUE_ID_BYTES = 128
MULTI_FLAT, MULTI_HIER, MULTI_LOCAL = 0, 1, 2          # allred_multi_plan.mode
TRANSPORT_RCCL, TRANSPORT_PEER, TRANSPORT_HOST = 0, 1, 2


class AllredError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = lib.allred_status_string(status).decode()
        super().__init__(f"{what}: {msg} ({status})" if what else f"{msg} ({status})")


def check(status: int, what: str = "") -> int:
    if status != OK:
        raise AllredError(status, what)
    return status


class Schedule(C.Structure):
    _fields_ = [
        ("algo", C.c_int32), ("side", C.c_int32), ("total", C.c_int32), ("steps", C.c_int32),
        ("partner", (C.c_int32 * MAX_STEPS) * MAX_NODES),
        ("send", (C.c_uint64 * MAX_STEPS) * MAX_NODES),
        ("recv", (C.c_uint64 * MAX_STEPS) * MAX_NODES),
        ("dirs", C.c_uint32 * MAX_NODES),
        ("tree_order", (C.c_uint8 * MAX_NODES) * MAX_NODES),
    ]


class PlanDesc(C.Structure):
    _fields_ = [
        ("algo", C.c_int32), ("variant", C.c_int32), ("exec", C.c_int32), ("side_length", C.c_int32),
        ("total_nodes", C.c_int32), ("device", C.c_int32), ("elems_per_rank", C.c_uint64),
        ("mem_accum", C.c_int32),
    ]


class Args(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "variant", "swing", "run_kernel", "side_length", "seed", "tiles", "error", "print_core",
        "bandwidth_optimal", "total_nodes", "exec", "round_mode", "num_tiles", "device", "mem_accum", "gpus")]


class Report(C.Structure):
    _fields_ = [
        ("mismatches", C.c_int64), ("max_error", C.c_float), ("device_seconds", C.c_double),
        ("e2e_seconds", C.c_double), ("bytes_per_rank", C.c_uint64), ("total_nodes", C.c_int32),
        ("launches", C.c_int32),
    ]


class DistDesc(C.Structure):
    _fields_ = [
        ("algo", C.c_int32), ("variant", C.c_int32), ("side_length", C.c_int32), ("total_nodes", C.c_int32),
        ("elems", C.c_uint64), ("local_ranks", C.c_int32), ("local_side", C.c_int32), ("local_algo", C.c_int32),
        ("channels", C.c_int32), ("mem_accum", C.c_int32),
    ]


class MultiPlan(C.Structure):
    _fields_ = [
        ("gpus", C.c_int32), ("local_ranks", C.c_int32), ("total_nodes", C.c_int32), ("variant", C.c_int32),
        ("mode", C.c_int32), ("print_core", C.c_int32), ("elems", C.c_uint64), ("validated_mask", C.c_uint64),
        ("desc", DistDesc),
    ]


class MultiOpts(C.Structure):
    _fields_ = [("transport", C.c_int32), ("share_device", C.c_int32), ("timeout_ms", C.c_int32),
                ("reserved", C.c_int32)]


class LaunchInfo(C.Structure):
    _fields_ = [("kernel", C.c_char * 64), ("grid", C.c_uint32), ("block", C.c_uint32), ("lds_bytes", C.c_uint32),
                ("regs", C.c_int32), ("resident_per_cu", C.c_int32), ("cus", C.c_int32), ("device", C.c_int32),
                ("reserved", C.c_int32)]


class Seg(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("bytes", C.c_uint64)]


EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(Seg), C.c_int, C.POINTER(Seg))

_P = C.c_void_p
_u16p = C.c_void_p
# (name, restype, argtypes) for every entry point declared in include/allred.h
SIGNATURES = [
    ("allred_status_string", C.c_char_p, [C.c_int]),
    ("allred_abi_version", C.c_int, []),
    ("allred_highest_power_of_two", C.c_int, [C.c_int]),
    ("allred_get_step_directions", C.c_uint32, [C.c_int, C.c_int]),
    ("allred_get_comm_partner_swing_2d", C.c_int, [C.c_int] * 5),
    ("allred_get_comm_partner_recdub_2d", C.c_int,
     [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint32), C.c_int]),
    ("allred_get_swing_block_comm_indexes", None,
     [C.c_int, C.c_int, C.POINTER(C.c_uint32), C.c_int, C.c_int, C.c_int]),
    ("allred_get_recdub_block_comm_indexes", None,
     [C.c_int, C.c_int, C.POINTER(C.c_uint32), C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint32)]),
    ("allred_normalize_tiles", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("allred_get_comm_partner_swing_1d", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("allred_get_comm_partner_recdub_1d", C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_uint32)]),
    ("allred_schedule_build", C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(Schedule)]),
    ("allred_lo_dag", C.c_int, [C.c_int, C.c_int, C.c_int, _P, C.c_size_t, C.POINTER(C.c_int)]),
    ("allred_steps_program", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, _P, C.c_size_t]),
    ("allred_random_bf16_vector", None, [C.c_size_t, C.c_int, C.c_int, C.c_int, _P]),
    ("allred_constant_bf16_vector", None, [C.c_size_t, C.c_float, _P]),
    ("allred_validate_result_vector", C.c_long,
     [_P, _P, _P, C.c_size_t, C.c_float, C.c_uint32, C.c_int, C.POINTER(C.c_float)]),
    ("allred_bf16_add", C.c_int, [_u16p, _u16p, C.c_size_t, _P]),
    ("allred_bf16_add_masked", C.c_int, [_u16p, _u16p, C.c_uint64, C.c_size_t, _P]),
    ("allred_tree_reduce", C.c_int, [_u16p, C.c_uint64, C.c_size_t, C.c_int, C.c_int, C.c_int, _u16p, _P]),
    ("allred_broadcast", C.c_int, [_u16p, C.c_uint64, C.c_size_t, C.c_int, _u16p, _P]),
    ("allred_preferred_rank_stride", C.c_uint64, [C.c_uint64]),
    ("allred_plan_create", C.c_int, [C.POINTER(PlanDesc), C.POINTER(_P)]),
    ("allred_plan_destroy", C.c_int, [_P]),
    ("allred_plan_workspace_bytes", C.c_size_t, [_P]),
    ("allred_plan_execute", C.c_int, [_P, _u16p, C.c_uint64, _P, _P]),
    ("allred_plan_launches", C.c_int, [_P]),
    ("allred_plan_stamp_words", C.c_uint64, [_P]),
    ("allred_plan_execute_profiled", C.c_int, [_P, _u16p, C.c_uint64, _P, _P, _P]),
    ("allred_plan_rank_zones", C.c_int, [_P, _P, _P, _P]),
    ("allred_tune_set", C.c_int, [C.c_char_p, C.c_int64]),
    ("allred_tune_get", C.c_int, [C.c_char_p, C.POINTER(C.c_int64)]),
    ("allred_last_launch", C.c_int, [C.POINTER(LaunchInfo)]),
    ("allred_args_parse", C.c_int, [C.c_int, C.POINTER(C.c_char_p), C.c_int, C.POINTER(Args)]),
    ("allred_run", C.c_int, [C.POINTER(Args), C.c_int, C.POINTER(Report)]),
    ("allred_comm_get_unique_id", C.c_int, [_P]),
    ("allred_comm_init", C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    ("allred_comm_init_all", C.c_int, [C.c_int, C.POINTER(C.c_int), C.POINTER(_P)]),
    ("allred_comm_destroy", C.c_int, [_P]),
    ("allred_dist_workspace_bytes", C.c_size_t, [C.POINTER(DistDesc)]),
    ("allred_dist_allreduce", C.c_int, [_P, C.POINTER(DistDesc), _u16p, _P, _P]),
    ("allred_dist_allreduce_pipelined", C.c_int, [_P, C.POINTER(DistDesc), _u16p, _P, _P]),
    ("allred_tree_broadcast_pipelined", C.c_int,
     [_u16p, _u16p, C.c_uint64, C.c_size_t, C.c_int, C.c_int, C.c_int, _u16p, _u16p, _P]),
    ("allred_dist_program_stats", C.c_int,
     [C.POINTER(DistDesc), C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("allred_dist_allreduce_host", C.c_int, [C.POINTER(DistDesc), C.c_int, _u16p, _u16p, EXCHANGE_FN, _P]),
    ("allred_comm_set_timeout", C.c_int, [_P, C.c_int]),
    ("allred_comm_wait", C.c_int, [_P, _P]),
    ("allred_comm_aborted", C.c_int, [_P]),
    ("allred_multi_plan_build", C.c_int, [C.POINTER(Args), C.c_int, C.POINTER(MultiPlan)]),
    ("allred_run_multi", C.c_int, [C.POINTER(Args), C.POINTER(MultiOpts), C.c_int, C.POINTER(Report), _u16p, _u16p]),
    ("allred_peer_create", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_uint64, C.POINTER(_P)]),
    ("allred_peer_handle", C.c_int, [_P, _P]),
    ("allred_peer_connect", C.c_int, [_P, _P]),
    ("allred_peer_connect_all", C.c_int, [C.c_int, C.POINTER(_P)]),
    ("allred_peer_allreduce", C.c_int, [_P, _u16p, C.c_uint64, C.c_int, C.c_int, C.c_int, _P, _P]),
    ("allred_peer_allreduce_pipelined2", C.c_int, [_P, _P, C.c_uint64, C.c_int, C.c_int, C.c_int, _P]),
    ("allred_peer_set_oneshot_max", C.c_int, [_P, C.c_uint64]),
    ("allred_peer_set_hier_ll", C.c_int, [_P, C.c_int]),
    ("allred_peer_set_max_groups", C.c_int, [_P, C.c_uint32]),
    ("allred_peer_set_lo_ll_max", C.c_int, [_P, C.c_uint64]),
    ("allred_peer_set_mem_ll_max", C.c_int, [_P, C.c_uint64]),
    ("allred_peer_set_sched_push", C.c_int, [_P, C.c_uint64]),
    ("allred_peer_dist_allreduce", C.c_int, [_P, C.POINTER(DistDesc), _u16p, _P, _P]),
    ("allred_peer_status", C.c_int, [_P, C.POINTER(C.c_uint32)]),
    ("allred_peer_clear_status", C.c_int, [_P]),
    ("allred_peer_check", C.c_int, [_P, _P]),
    ("allred_peer_destroy", C.c_int, [_P]),
]
PEER_HANDLE_BYTES = 256
PEER_MAX_WINDOW_BYTES = 1 << 30   # allred_peer_create rejects larger windows (allred.h)
PEER_TIMEOUT, PEER_WIN_CACHED, PEER_FLAGS_CACHED = 0x1, 0x100, 0x200   # allred_peer_status bits

for _name, _res, _args in SIGNATURES:  # noqa: E305
    if "ALLRED_LIB_PATH" in os.environ and not hasattr(lib, _name):
        continue  # an older build under A/B may predate a later entry point
    _f = getattr(lib, _name)  # AttributeError here = the library lacks a declared symbol
    _f.restype = _res
    _f.argtypes = _args

if "ALLRED_LIB_PATH" not in os.environ and lib.allred_abi_version() != ABI_VERSION:
    raise ImportError(f"{LIB_PATH}: ABI {lib.allred_abi_version()}, this package expects {ABI_VERSION}: rebuild it")
