"""The C-ABI boundary without a GPU: every symbol include/allred.h declares is
exported, the host-only entry points behave like the reference's, and the
source-compatible allred_helper.hpp compiles, links and runs."""
import os
import re
import subprocess
import sys

import ctypes as C

import numpy as np
import pytest

import oracle
import tenstorrentallreduce_amd as t
from tenstorrentallreduce_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "allred.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(allred_\w+)\s*\(", src))
    return sorted(n for n in names if not n.endswith("_fn"))


def test_every_declared_symbol_is_exported_and_bound():
    names = declared_functions()
    assert len(names) >= 30
    bound = {n for n, _, _ in _lib.SIGNATURES}
    for n in names:
        assert hasattr(_lib.lib, n), n
        assert n in bound, f"{n} declared in allred.h but not bound in _lib.SIGNATURES"
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}\b", nm), n


def test_header_constants_match_python_bindings():
    src = open(os.path.join(ROOT, "include", "allred.h")).read()
    defines = dict(re.findall(r"#define\s+(ALLRED_\w+)\s+(0x[0-9a-fA-F]+|\d+)u?\b", src))
    assert int(defines["ALLRED_PEER_HANDLE_BYTES"], 0) == _lib.PEER_HANDLE_BYTES
    assert int(defines["ALLRED_PEER_TIMEOUT"], 0) == t.PEER_TIMEOUT
    assert int(defines["ALLRED_ABI_VERSION"], 0) == _lib.ABI_VERSION
    assert (int(defines["ALLRED_ACC_FP32"]), int(defines["ALLRED_ACC_BF16"])) == (t.ACC_FP32, t.ACC_BF16)


def test_status_strings():
    assert _lib.lib.allred_abi_version() == _lib.ABI_VERSION == 7
    for st in range(0, -8, -1):
        assert _lib.lib.allred_status_string(st)


REF_DEFAULTS = dict(swing=0, run_kernel=0, side_length=1, seed=0, tiles=1, error=1, print_core=0, bandwidth_optimal=0,
                    exec=t.EXEC_FUSED, device=-1, mem_accum=t.ACC_FP32)


@pytest.mark.parametrize("argv,want", [
    ([], {}),
    (["1"], {"swing": 1}),
    (["2"], {"swing": 0}),                                     # only == 1 selects Swing
    (["1", "1", "8", "13", "5", "32", "0", "1"],
     {"swing": 1, "run_kernel": 1, "side_length": 8, "seed": 13, "tiles": 5, "error": 32, "bandwidth_optimal": 1,
      "num_tiles": 320, "total_nodes": 64}),
    (["0", "1", "5", "-1", "0", "32", "3", "0"],               # side 5 -> 4; tiles 0 -> 1
     {"run_kernel": 1, "side_length": 4, "seed": -1, "tiles": 1, "error": 32, "print_core": 3, "num_tiles": 1}),
    (["0", "1", "100", "7", "65", "1", "0", "0"], {"run_kernel": 1, "side_length": 8, "seed": 7, "tiles": 65,
                                                  "num_tiles": 128}),
    (["1", "1", "8", "13", "3", "32", "0", "0"],               # LO: next power of two
     {"swing": 1, "run_kernel": 1, "side_length": 8, "seed": 13, "tiles": 3, "error": 32, "num_tiles": 4}),
    (["0", "1", "4", "13", "40", "32", "0", "1", "8"],         # rank-count extension: 4x2 grid
     {"run_kernel": 1, "side_length": 4, "seed": 13, "tiles": 40, "error": 32, "bandwidth_optimal": 1,
      "total_nodes": 8, "num_tiles": 320}),
    ([" 12abc"], {"swing": 0}),                                 # std::stoi reads the leading integer
])
def test_args_parse_like_allredconfig(argv, want):
    a = t.parse_args(["allred_BO_2D", *argv], t.BO)
    exp = dict(REF_DEFAULTS)
    exp.update(want)
    for k, v in exp.items():
        assert getattr(a, k) == v, (k, getattr(a, k), v)


def test_args_parse_variants():
    # allred_mem_2D: large_buffer = true (allred_mem_2D.cpp:15); args 7/8 ignored
    a = t.parse_args(["allred_mem_2D", "1", "1", "8", "13", "5", "32", "9", "0"], t.MEM)
    assert a.num_tiles == 320 and a.print_core == 0
    a = t.parse_args(["allred_LO_2D", "1", "1", "8", "13", "5", "32"], t.LO)
    assert a.num_tiles == 8


def test_args_parse_extension_envs(monkeypatch):
    """Extensions never change a reference invocation: the one-pass form is the
    default (ALLRED_EXEC=steps opts into the step structure), ALLRED_DEVICE
    names the HIP device (the reference's CreateDevice(0), allred_BO_2D.cpp:8),
    ALLRED_MEM_ACC=bf16 the reference's bf16 dest accumulation."""
    argv = ["allred_mem_2D", "1", "1", "8", "13", "5", "32"]
    monkeypatch.setenv("ALLRED_EXEC", "steps")
    monkeypatch.setenv("ALLRED_DEVICE", "3")
    monkeypatch.setenv("ALLRED_MEM_ACC", "bf16")
    a = t.parse_args(argv, t.MEM)
    assert (a.exec, a.device, a.mem_accum) == (t.EXEC_STEPS, 3, t.ACC_BF16)
    monkeypatch.setenv("ALLRED_DEVICE", "x")
    with pytest.raises(t.AllredError):
        t.parse_args(argv, t.MEM)


def test_tune_entry_point():
    """allred_tune_set / allred_tune_get: the one switch for bit-identical kernel forms."""
    assert t.tune("steps_form") == 0 and t.tune("lo_tree") == 1 and t.tune("fused_form") == 0
    with t.tuned(steps_form=1, lo_dag_min_tiles=1024):
        assert t.tune("steps_form") == 1 and t.tune("lo_dag_min_tiles") == 1024
    assert t.tune("steps_form") == 0 and t.tune("lo_dag_min_tiles") == 256
    with pytest.raises(t.AllredError):
        t.tune("no_such_key")
    with pytest.raises(t.AllredError):
        t.tune("fused_form", 9)          # out of range
    assert t.tune("fused_form") == 0
    # the schedule form's grid: auto by default, at most 5 workgroups per CU
    assert t.tune("steps_groups") == 0
    with t.tuned(steps_groups=4):
        assert t.tune("steps_groups") == 4
    with pytest.raises(t.AllredError):
        t.tune("steps_groups", 6)
    for v in (1, 2):   # documented values are 0 (auto), 3, 4, 5 only
        with pytest.raises(t.AllredError):
            t.tune("steps_groups", v)
    assert t.tune("steps_groups") == 0
    # round-4 keys: defaults are the product forms / no fault injection
    assert (t.tune("rccl_fault"), t.tune("multi_fault")) == (0, 0)
    with pytest.raises(t.AllredError):
        t.tune("rccl_fault", 8)
    # round 5: the flag hand-off forms are gone with their key (the trimmed table); peer_fence
    # (release / acquire fences around every cross-GPU hand-off) is off by default, 0 / 1 only
    with pytest.raises(t.AllredError):
        t.tune("hier_handoff")
    assert t.tune("peer_fence") == 0
    with t.tuned(peer_fence=1):
        assert t.tune("peer_fence") == 1
    with pytest.raises(t.AllredError):
        t.tune("peer_fence", 2)
    # k_hier_ws: half tiles per reducing wave by default (8 / 16 / 32 columns only), loads one
    # tile ahead (1 / 2)
    assert (t.tune("hier_ws_cols"), t.tune("hier_ws_ahead")) == (16, 1)
    for v in (8, 32):
        with t.tuned(hier_ws_cols=v):
            assert t.tune("hier_ws_cols") == v
    for key, bad in (("hier_ws_cols", 12), ("hier_ws_cols", 64), ("hier_ws_ahead", 0), ("hier_ws_ahead", 3)):
        with pytest.raises(t.AllredError):
            t.tune(key, bad)
    assert t.tune("hier_ws_cols") == 16


def test_mem_program_stats_one_rank_has_no_launch():
    """mem_2D over RCCL on a 1-rank grid: no exchange, so no sum kernel either."""
    st = t.dist_program_stats(t.dist_desc(t.SWING, t.MEM, 1, 1, 64), 0)
    assert (st["steps"], st["add_launches"]) == (0, 0)
    st = t.dist_program_stats(t.dist_desc(t.SWING, t.MEM, 4, 8, 8 * 8 * 4), 3)
    assert (st["steps"], st["add_launches"]) == (2, 1)


def test_tune_env_is_read_at_load():
    code = ("import sys; sys.path.insert(0, %r); import tenstorrentallreduce_amd as t;"
            "print(t.tune('steps_form'), t.tune('lo_dag_place'), t.tune('pipe_grid'))" % ROOT)
    env = dict(os.environ, ALLRED_TUNE="steps_form=1,lo_dag_place=0,bogus=3,pipe_grid=99999999")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env).stdout.split()
    assert out == ["1", "0", "0"]   # out-of-range and unknown keys are ignored
    env = dict(os.environ, ALLRED_TUNE="steps_groups=3")
    out = subprocess.run([sys.executable, "-c", code.replace("t.tune('steps_form'), ", "t.tune('steps_groups'), ")],
                         capture_output=True, text=True, env=env).stdout.split()
    assert out[0] == "3"


def test_peer_window_limit_without_gpu():
    """allred_peer_create rejects any window over 1 GiB (a ~2 GiB IPC export hung
    the peer's hipIpcOpenMemHandle, profiles/r01_peer_open_probe_2gib_hang.txt)
    before any HIP call, so the limit holds on a machine without a GPU."""
    import ctypes as C
    h = C.c_void_p()
    for elems in ((1 << 29) + 1, 1 << 30, 3 << 29):
        assert _lib.lib.allred_peer_create(2, 0, -1, elems, C.byref(h)) == _lib.ERR_ARG
        assert not h.value
    assert _lib.PEER_MAX_WINDOW_BYTES == 1 << 30


@pytest.mark.parametrize("algo,variant,chans", [(t.SWING, t.BO, 7), (t.RECDUB, t.BO, 7), (t.RECDUB, t.BO, 1),
                                                (t.SWING, t.LO, 1), (t.SWING, t.BO, 3)])
def test_dist_program_one_add_launch_per_step(algo, variant, chans):
    """The RCCL program (dist.cpp) adds every received run of every link-spreading
    channel of a step in ONE launch: 8 ranks (4x2), BO = 3 reduce-scatter steps
    with adds + 3 all-gather steps without; LO = 3 add steps."""
    n = 8 * 8 * 7 * 640 * 4
    desc = t.dist_desc(algo, variant, 4, 8, n, channels=chans)
    for rank in range(8):
        st = t.dist_program_stats(desc, rank)
        if variant == t.BO:
            assert st["steps"] == 6 and st["add_launches"] == 3, st
        else:
            assert st["steps"] == 3 and st["add_launches"] == 3, st
        assert st["segments"] >= st["steps"] * 2 * (chans if variant == t.BO else 1)


@pytest.mark.parametrize("bad", [["x"], ["1", "1", "abc"], ["1", "1", "8", "13", "99999999999"]])
def test_args_parse_rejects_junk_like_stoi(bad):
    with pytest.raises(t.AllredError):
        t.parse_args(["allred_BO_2D", *bad], t.BO)


def test_validate_matches_oracle_counts():
    n = 4096
    s0 = t.random_bf16_vector(2 * n, 13)
    s1 = t.random_bf16_vector(2 * n, 14)
    _, _, ranks = oracle.reference_inputs(8, 64, n, 13)
    good = ranks[0].copy()
    oracle.allreduce("bo", oracle.SWING, 8, [r.copy() for r in ranks], 64)
    rs = [r.copy() for r in ranks]
    oracle.allreduce("bo", oracle.SWING, 8, rs, 64)
    res = rs[0].view(np.uint32)
    assert t.validate_result_vector(res, s0, s1, n // 2, 32, 64)[0] == 0
    assert oracle.validate(res, s0, s1, 64, 32)[0] == 0
    bad = rs[0].copy()
    bad[::97] ^= 0x0100  # perturb exponent bits of some elements
    b1, m1 = t.validate_result_vector(bad.view(np.uint32), s0, s1, n // 2, 32, 64)
    b2, m2 = oracle.validate(bad.view(np.uint32), s0, s1, 64, 32)
    assert b1 == b2 > 0
    del good


def test_validate_prints_reference_messages():
    code = (
        "import sys; sys.path.insert(0, %r); import numpy as np, tenstorrentallreduce_amd as t;"
        "a = t.constant_bf16_vector(2048, 1.0); r = t.constant_bf16_vector(2048, 4.0);"
        "t.validate_result_vector(r, a, a, 512, 1, 4, True);"
        "w = t.constant_bf16_vector(2048, 5.0); t.validate_result_vector(w, a, a, 512, 0, 4, True)" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True).stdout
    assert out.startswith("All values match!\n")
    assert "Mismatch at index 0:\n  Expected: 4\n  Actual  : 5\n" in out
    assert "Total matches: 0" in out and "Max error: 1.000000" in out and "Mismatch blocks: 0 " in out


def test_allred_helper_hpp_compiles_and_runs(tmp_path):
    """A reference-style host program against the source-compatible header."""
    prog = tmp_path / "p.cpp"
    prog.write_text(r'''
#include "allred_helper.hpp"
#include <cstdio>
int main() {
    uint32_t dirs = 0;
    int p = get_comm_partner_recdub_2D(0, 0, true, 1, dirs, 8);
    uint32_t blocks[2] = {0, 0};
    get_swing_block_comm_indexes(1, 1, blocks, false, 8, 64);
    std::vector<uint32_t> a(256, 0x3f803f80u), r(256, 0x40803f80u | 0x00004080u);
    for (auto& x : r) x = 0x40804080u;
    validate_result_vector(r, a, a, 256, 0, 4);
    std::printf("%d %u %u %u %d\n", p, dirs, blocks[0], blocks[1], highest_power_of_two(6));
    return 0;
}
''')
    exe = tmp_path / "p"
    lib_dir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", f"-I{ROOT}/include", str(prog), "-o", str(exe), f"-L{lib_dir}", "-lallred",
                    f"-Wl,-rpath,{lib_dir}", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    assert out[0] == "All values match!"
    p, dirs, b0, b1, hp = out[1].split()
    assert (int(p), int(dirs), int(hp)) == (1, 1, 4)
    assert int(b0) | (int(b1) << 32) == t.get_swing_block_comm_indexes(1, 1, 0, False, 8, 64)


def test_gpus_extension_parse_and_validation_without_gpu(monkeypatch):
    """ALLRED_GPUS / argv[10] (the reference's argv across a node's GPUs): parsed
    like the other extensions, and a rank split that cannot work (G not a power
    of two, G not dividing the rank count, mem_2D with several ranks on several
    GPUs) is refused with ALLRED_ERR_ARG / _UNSUPPORTED before any HIP call."""
    a = t.parse_args(["allred_BO_2D", "0", "1", "4", "13", "40", "32", "0", "1", "8", "4"], t.BO)
    assert (a.total_nodes, a.gpus) == (8, 4)
    monkeypatch.setenv("ALLRED_GPUS", "2")
    a = t.parse_args(["allred_BO_2D", "0", "1", "4", "13", "40", "32", "0", "1"], t.BO)
    assert a.gpus == 2
    monkeypatch.delenv("ALLRED_GPUS")
    assert t.parse_args(["allred_BO_2D", "0", "1", "4"], t.BO).gpus == 0
    with pytest.raises(t.AllredError):
        t.parse_args(["allred_BO_2D", "0", "1", "4", "13", "40", "32", "0", "1", "8", "x"], t.BO)
    for argv, variant, want in (
            (["allred_BO_2D", "0", "1", "4", "13", "40", "32", "0", "1", "8", "3"], t.BO, _lib.ERR_ARG),
            (["allred_BO_2D", "0", "1", "2", "13", "40", "32", "0", "1", "4", "8"], t.BO, _lib.ERR_ARG),
            (["allred_mem_2D", "1", "1", "4", "13", "40", "32", "0", "0", "8", "2"], t.MEM, _lib.ERR_UNSUPPORTED)):
        a = t.parse_args(argv, variant)
        r = _lib.Report()
        assert _lib.lib.allred_run(C.byref(a), 0, C.byref(r)) == want, argv


# the whole tune table (tune.cpp kKeys, allred.h §Tuning): every key readable, the retired ones gone
TUNE_KEYS = ("fused_form", "lo_tree", "lo_dag", "lo_dag_place", "lo_dag_min_tiles", "mem_reduce_lds", "steps_form",
             "pipe_grid", "lo_dag_reg", "lo_dag_reg_min_tiles", "check", "fused_chunk_tiles", "lo_tree_min_tiles",
             "tree_bcast_lag", "tree_bcast_bal", "steps_groups", "rccl_fault", "multi_fault", "steps_tab",
             "steps_early", "peer_fence", "hier_ws_ahead", "hier_ws_cols")
RETIRED_KEYS = ("hier_handoff", "hier_x2_tail", "hier_x_lag", "hier_x_chunked", "hier_x_rearly", "hier_x_latepoll")


def test_tune_table_is_the_product_forms_only():
    """ABI 7 (round 6): the keys that served only the retired hierarchical forms (k_hier_ll,
    the one-deep pipeline k_hier_x, k_hier_x2's other placements) are gone; the table is at
    most 24 keys, each with its documented default."""
    assert len(TUNE_KEYS) <= 24
    for key in TUNE_KEYS:
        t.tune(key)   # readable (raises if unknown)
    for key in RETIRED_KEYS:
        with pytest.raises(t.AllredError):
            t.tune(key)
    hdr = open(os.path.join(ROOT, "include", "allred.h")).read()
    tune_doc = hdr[hdr.index("Tuning: the one entry point"):hdr.index("int allred_tune_set")]
    for key in TUNE_KEYS:
        assert f" {key} " in tune_doc, f"{key} undocumented in allred.h"
    for key in RETIRED_KEYS:
        assert f" {key} " not in tune_doc, key


def test_ctypes_structures_match_the_header_layout(tmp_path):
    """Every struct _lib.py mirrors has the header's size and field offsets (a C program
    compiled against include/allred.h prints them): a binding that drops or reorders a
    field — e.g. a PlanDesc without mem_accum — reads past the caller's struct."""
    structs = {"allred_plan_desc": _lib.PlanDesc, "allred_args": _lib.Args, "allred_report": _lib.Report,
               "allred_dist_desc": _lib.DistDesc, "allred_multi_plan": _lib.MultiPlan,
               "allred_multi_opts": _lib.MultiOpts, "allred_launch_info": _lib.LaunchInfo,
               "allred_seg": _lib.Seg, "allred_schedule": _lib.Schedule}
    lines = []
    for cname, py in structs.items():
        lines.append(f'    std::printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'    std::printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    prog = tmp_path / "layout.cpp"
    prog.write_text('#include <cstddef>\n#include <cstdio>\n#include "allred.h"\nint main() {\n' + "\n".join(lines) +
                    "\n    return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        cname, field, value = line.split()
        got[(cname, field)] = int(value)
    for cname, py in structs.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)
