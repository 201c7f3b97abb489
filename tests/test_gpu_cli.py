"""The reference's executables and invocations, unchanged, on the MI355X build
(README.md:23-45, python/timing_taker.py:60-65).  Pass signal = the
reference's own stdout line "All values match!" (allred_helper.cpp:75)."""
import json
import os

import pytest

import tenstorrentallreduce_amd as t

pytestmark = pytest.mark.gpu


def run(binary, argv, **env):
    p = t.run_cli(binary, argv, env={"ALLRED_REPORT": "1", "ALLRED_CHECK_ALL": "1", **env})
    assert p.returncode == 0, p.stderr
    rep = json.loads(p.stderr.strip().splitlines()[-1])
    return p.stdout, rep


@pytest.mark.parametrize("argv", [
    ["0", "1", "2", "-1", "1", "32", "0", "0"],      # BASELINE config 1: 2x2 RecDub LO, 1 tile, all ones
    ["1", "1", "8", "13", "5", "32", "0", "1"],      # BASELINE config 2: 8x8 Swing BO, 5 tiles
    ["0", "1", "8", "13", "5", "32", "0", "1"],      # 8x8 RecDub BO
    ["1", "1", "8", "13", "320", "32", "0", "0"],    # LO 640 kB
    ["0", "1", "8", "13", "3", "32", "0", "0"],      # LO 8 kB (LOO-sized)
    ["1", "1", "4", "13", "2", "32", "3", "1"],      # 4x4 BO
])
def test_allred_BO_2D(argv):
    out, rep = run("allred_BO_2D", argv)
    assert "All values match!" in out
    assert rep["mismatches"] == 0


@pytest.mark.parametrize("exec_mode", ["steps", "fused"])
@pytest.mark.parametrize("size", [1, 2, 4, 8, 16, 32, 64, 128, 192, 256, 320])
@pytest.mark.parametrize("swing", ["0", "1"])
def test_timing_taker_lo_sweep(swing, size, exec_mode):
    """python/timing_taker.py:125,172-176 LO sizes: <bin> <swing> 1 8 13 <size> 32 0 0."""
    out, rep = run("allred_BO_2D", [swing, "1", "8", "13", str(size), "32", "0", "0"], ALLRED_EXEC=exec_mode)
    assert "All values match!" in out


@pytest.mark.parametrize("size", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("binary", ["allred_BO_2D", "allred_mem_2D"])
def test_timing_taker_bo_mem_sweep(binary, size):
    argv = ["1", "1", "8", "13", str(size), "32"] + (["0", "1"] if binary == "allred_BO_2D" else [])
    out, rep = run(binary, argv)
    assert "All values match!" in out
    assert rep["bytes_per_rank"] == size * 128 * 1024


@pytest.mark.parametrize("bo", ["0", "1"])
def test_exact_under_rne_ctor(bo):
    """With the RNE bfloat16(float) ctor for inputs and expected values, the
    engine's result equals the reference's expected vector exactly (ERROR 0):
    RNE(a+b) * N/2 == RNE((a+b) * N/2)."""
    out, rep = run("allred_BO_2D", ["1", "1", "8", "13", "5", "0", "0", bo], ALLRED_BF16_ROUND="rne")
    assert "All values match!" in out and rep["max_error"] == 0


def test_allred_LO_2D_legacy():
    out, rep = run("allred_LO_2D", ["1", "1", "8", "13", "4", "32"])
    assert "All values match!" in out


def test_rank_count_extension_rectangular_grid():
    # 8 ranks on a 4x2 grid (the 8-GPU mapping), via the trailing extension argument
    out, rep = run("allred_BO_2D", ["1", "1", "4", "13", "40", "32", "0", "1", "8"])
    assert "All values match!" in out and rep["ranks"] == 8 and rep["bytes_per_rank"] == 655360


def test_mismatch_report_when_kernel_not_run():
    """RUN_KERNEL = 0 still reads back and validates (allred_helper.hpp:85-93):
    the inputs are not reduced, so the reference's mismatch report appears."""
    p = t.run_cli("allred_BO_2D", ["1", "0", "2", "13", "1", "32", "0", "1"])
    assert p.returncode == 0
    assert "Mismatch at index 0:" in p.stdout and "Max error:" in p.stdout


def test_bad_argument_fails_like_stoi():
    p = t.run_cli("allred_BO_2D", ["x"])
    assert p.returncode != 0 and "stoi" in p.stderr


@pytest.mark.parametrize("e2e", ["zerocopy", "dma"])
def test_config2_fused_both_end_to_end_modes(e2e):
    """BASELINE config 2 through the reference CLI with the fused pass, the buckets
    starting and ending in pinned host memory: read in place over PCIe
    (zero-copy, the default) and staged by one DMA each way."""
    out, rep = run("allred_BO_2D", ["1", "1", "8", "13", "5", "32", "0", "1"], ALLRED_EXEC="fused", ALLRED_E2E=e2e)
    assert "All values match!" in out
    assert rep["mismatches"] == 0


@pytest.mark.parametrize("argv", [["1", "1", "8", "13", "5", "32", "0", "1"],      # config 2, 640 kB
                                  ["0", "1", "8", "13", "40", "0", "63", "1"]])  # RecDub, 5 MiB per rank
@pytest.mark.parametrize("chunks", ["default", "1", "2", "5", "10", "16", "3"])
def test_dma_end_to_end_chunked_is_exact(argv, chunks):
    """The DMA end-to-end form over column chunks: chunk c's 2D H2D, its fused
    pass and its 2D D2H on three streams, overlapping across chunks — 8 by
    default, or ALLRED_E2E_CHUNKS.  Every rank equals the reference's expected value at ERROR 0
    (RNE ctor, ALLRED_CHECK_ALL).  3 chunks do not divide the bucket's blocks:
    the one-copy form runs instead (still exact)."""
    argv = list(argv)
    argv[5] = "0"
    env = {} if chunks == "default" else {"ALLRED_E2E_CHUNKS": chunks}
    out, rep = run("allred_BO_2D", argv, ALLRED_EXEC="fused", ALLRED_E2E="dma", ALLRED_BF16_ROUND="rne", **env)
    assert out.strip() == "All values match!", out
    assert rep["mismatches"] == 0 and rep["e2e_s"] > rep["device_s"] > 0


@pytest.mark.parametrize("ratio,launches", [("0", 1), ("1e9", 8), ("default", None)])
def test_dma_strided_copy_probe_both_outcomes(ratio, launches):
    """The chunk-or-not decision of the DMA end-to-end form (engine.cpp): with no
    ALLRED_E2E_CHUNKS, allred_run times one strided (2D) and one plain device-to-host
    copy of a chunk in its untimed warm-up and keeps the 8 column chunks only where
    the strided one takes at most ALLRED_E2E_STRIDED_RATIO (default 1.5) x the plain
    one's time — some boxes move 2D copies at ~23 GB/s against ~52 for plain ones
    (DESIGN.md §6).  Ratio 0 forces the one-copy outcome (one pass: 1 launch), a huge
    ratio the chunked one (8 passes); the default takes whichever this box's probe
    picks.  Every outcome: "All values match!" on every rank at ERROR 0 (RNE ctor).
    The reference's own H2D / D2H around the run: allred_helper.cpp:287-288,
    allred_helper.hpp:92."""
    env = {} if ratio == "default" else {"ALLRED_E2E_STRIDED_RATIO": ratio}
    out, rep = run("allred_BO_2D", ["1", "1", "8", "13", "5", "0", "0", "1"], ALLRED_EXEC="fused", ALLRED_E2E="dma",
                   ALLRED_BF16_ROUND="rne", **env)
    assert out.strip() == "All values match!", out
    assert rep["mismatches"] == 0 and rep["e2e_s"] > rep["device_s"] > 0
    if launches is not None:
        assert rep["launches"] == launches, rep
    else:
        assert rep["launches"] in (1, 8), rep


@pytest.mark.parametrize("exec_mode", ["steps", "fused"])
def test_allredconfig_runprogram_cpp_program(exec_mode):
    """A reference-style C++ program against include/allred_helper.hpp alone
    (bin/allred_config_main: AllredConfig(argc, argv, ALLRED_BO, device 0)
    .RunProgram(), the shape of allred_BO_2D.cpp:7-215) on BASELINE config 2;
    its pass signal is the reference's own stdout line."""
    import os
    import subprocess
    exe = os.path.join(t._lib.BIN_DIR, "allred_config_main")
    env = dict(os.environ, ALLRED_EXEC=exec_mode, ALLRED_CHECK_ALL="1")
    p = subprocess.run([exe, "0", "1", "1", "8", "13", "5", "32", "0", "1"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.startswith("All values match!\n"), p.stdout
    assert "ranks 64 tiles 320 device 0" in p.stdout


def test_cli_default_is_the_fused_form():
    """The one-pass form is the reference CLI's default (bit-identical to the
    step structure, which ALLRED_EXEC=steps keeps): one launch per allreduce."""
    _, rep = run("allred_BO_2D", ["1", "1", "8", "13", "5", "32", "0", "1"])
    assert rep["launches"] == 1 and rep["mismatches"] == 0
    _, rep = run("allred_BO_2D", ["1", "1", "8", "13", "5", "32", "0", "1"], ALLRED_EXEC="steps")
    assert rep["launches"] == 1 and rep["mismatches"] == 0   # the schedule form is one persistent launch too


@pytest.mark.parametrize("argv,bo", [(["1", "1", "8", "13", "5", "32", "0", "1"], True),
                                     (["0", "1", "8", "13", "5", "32", "0", "1"], True),
                                     (["1", "1", "8", "13", "16", "32", "0", "0"], False)])
def test_profile_log_per_rank_zones(argv, bo, tmp_path):
    """ALLRED_PROFILE_LOG (the reference's TT_METAL_DEVICE_PROFILER=1 +
    profile_log_device.csv): the schedule form stamps every unit on the device
    (s_memrealtime), the library turns them into each rank's ALL_RED_LOOP zone,
    and the reference's analysis (tools/profile_analyzer.py) reads the CSV:
    64 cores, each zone non-empty, every start before every rank's end."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from profile_analyzer import analyze, normalized
    log = tmp_path / "profile_log_device.csv"
    out, rep = run("allred_BO_2D", argv, ALLRED_EXEC="steps", ALLRED_E2E="dma", ALLRED_PROFILE_LOG=str(log))
    assert "All values match!" in out
    stats = analyze(str(log))
    assert stats["cores"] == 64 and stats["min"] > 0
    norm = normalized(str(log))
    assert len(norm) == 64
    starts = [s for s, _ in norm.values()]
    ends = [e for _, e in norm.values()]
    assert min(starts) == 0 and max(starts) < min(ends)
    # zones lie inside the event-timed device interval (100 MHz ticks), with slack for clock skew
    assert max(ends) <= rep["device_s"] * 1e8 * 1.2 + 200


@pytest.mark.parametrize("binary,argv", [
    ("allred_BO_2D", ["0", "1", "4", "13", "40", "32", "0", "1"]),   # BASELINE config 3's invocation (4x2 RecDub BO)
    ("allred_BO_2D", ["1", "1", "4", "13", "40", "32", "0", "1"]),   # Swing BO, the config-4 program at 640 kB
    ("allred_BO_2D", ["1", "1", "4", "13", "16", "32", "0", "0"]),   # config 5's Swing LO (32 kB)
    ("allred_BO_2D", ["1", "1", "8", "13", "5", "32", "0", "1"]),    # config 2's 64 ranks
    ("allred_mem_2D", ["1", "1", "4", "13", "40", "32"]),            # mem_2D, all ranks on the one GPU
    ("allred_LO_2D", ["0", "1", "4", "13", "4", "32"]),
])
@pytest.mark.parametrize("via", ["env", "argv"])
def test_gpus_extension_one_gpu(binary, argv, via):
    """The multi-GPU mode of the reference executables (ALLRED_GPUS or argv[10]:
    one host thread and one RCCL rank per GPU, ncclCommInitAll) at G = 1: the
    rank grid's ranks all on GPU 0 (the local tree of the reference's own
    (side, total) grid, a 1-rank RCCL program, the broadcast), every rank checked
    with the reference's validate_result_vector; exact (error 0) under the RNE
    ctor, where the result is RNE(a+b) * N/2 for every tree."""
    nodes = "8" if argv[2] == "4" else "64"
    env = {"ALLRED_NODES": nodes, "ALLRED_BF16_ROUND": "rne"}
    args = list(argv)
    args[5] = "0"   # error 0
    if via == "env":
        env["ALLRED_GPUS"] = "1"
    else:
        args = args + ["0"] * (8 - len(args)) + [nodes, "1"]
    out, rep = run(binary, args, **env)
    assert "All values match!" in out, out
    assert rep["mismatches"] == 0 and rep["max_error"] == 0 and rep["ranks"] == int(nodes)
    assert rep["launches"] == -1 and rep["device_s"] > 0


def test_gpus_extension_rejects_more_gpus_than_visible():
    import torch
    p = t.run_cli("allred_BO_2D", ["0", "1", "4", "13", "40", "32", "0", "1"],
                  env={"ALLRED_NODES": "8", "ALLRED_GPUS": str(2 * max(1, torch.cuda.device_count()))})
    assert p.returncode == 1 and "argument" in p.stderr.lower()


def test_comm_init_all_mem_one_rank():
    """allred_comm_init_all on one device and the mem_2D variant of the RCCL
    program (local_ranks == 1) on a 1-rank grid: the bucket comes back unchanged."""
    import numpy as np
    import torch
    comms = t.Comm.init_all([0])
    n = 8 * 1024
    x = torch.randint(0x3F80, 0x42C8, (n,), dtype=torch.int32).to(torch.int16).to("cuda:0")
    want = x.clone()
    desc = t.dist_desc(t.SWING, t.MEM, 1, 1, n)
    ws = torch.empty(t.dist_workspace_bytes(desc), dtype=torch.uint8, device="cuda:0")
    t.dist_allreduce(comms[0], desc, x.data_ptr(), ws.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert torch.equal(x, want)
    comms[0].close()
