"""The RCCL half of tests/test_gpu_multidevice.py on CPU: the bodies of
test_rccl_programs_across_gpus, test_rccl_pipelined_across_gpus and
test_config4_one_gib_over_rccl_across_gpus with the RCCL exchange replaced by
the library's host twin of the same per-rank program (allred_dist_allreduce_host
over gloo, world 2 / 4 / 8) — the same cases, inputs and expectation code
(tests/multi_cases.py), the buckets reduced where noted.  RCCL refuses two ranks
on one device, so those GPU cases could never be rehearsed; with their
expectations proven here, a red case on the first multi-GPU box points at the
product, not at the test.  (The reference validates every run:
allred_helper.hpp:84-96 -> validate_result_vector, allred_helper.cpp:18-120.)"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def gloo_exchange(peer, sends, recvs):
    reqs = [dist.isend(torch.from_numpy(v), peer, tag=i) for i, v in enumerate(sends)]
    reqs += [dist.irecv(torch.from_numpy(v), peer, tag=i) for i, v in enumerate(recvs)]
    for r in reqs:
        r.wait()


def worker(rank, world, port, q, which):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, ROOT)
        sys.path.insert(0, HERE)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import tenstorrentallreduce_amd as t
        import multi_cases as mc
        import test_dist_host as tdh
        dist.init_process_group("gloo", rank=rank, world_size=world)
        side, total = tdh.GRIDS[world]
        fails = []

        def host(desc, buf, local):
            scratch = np.zeros(max(2 * int(desc.elems), t.dist_workspace_bytes(desc) // 2 + 8), dtype=np.uint16)
            t.dist_allreduce_host(desc, rank, buf, scratch, gloo_exchange)

        if which == "programs":   # test_rccl_programs_across_gpus: every case, twice, then mem_2D fp32 / bf16
            for ci, (variant, algo, local, chans, n) in enumerate(mc.rccl_cases(world)):
                desc = mc.rccl_case_desc(world, variant, algo, local, chans, n)
                for rep in range(2):
                    data = mc.rccl_case_inputs(world, local, n, ci, rep)
                    buf = np.concatenate(data[rank]).astype(np.uint16)
                    host(desc, buf, local)
                    want = mc.rccl_case_expected(world, variant, algo, local, chans, n, data)[rank]
                    if not np.array_equal(buf, want):
                        fails.append((variant, algo, local, chans, n, rep, int((buf != want).sum())))
            for acc in (t.ACC_FP32, t.ACC_BF16):
                n = 8 * total * 640
                desc = t.dist_desc(t.SWING, t.MEM, side, total, n, mem_accum=acc)
                data = mc.rccl_mem_inputs(world, acc, n)
                buf = data[rank].copy()
                host(desc, buf, 1)
                want = mc.rccl_mem_expected(world, acc, data)[rank]
                if not np.array_equal(buf, want):
                    fails.append(("mem", acc, int((buf != want).sum())))
        elif which == "pipelined":   # test_rccl_pipelined_across_gpus: 64 local ranks per GPU, K = 3 buckets
            # (the GPU test's 327,680 elements per rank reduced to 8 x total x 64; the pipelined
            # form's bits per bucket are allred_dist_allreduce's, which the host twin runs)
            n, local, K = 8 * total * 64, 64, 3
            desc = t.dist_desc(t.SWING, t.BO, side, total, n, local_ranks=local, local_side=8, local_algo=t.SWING)
            data = mc.pipelined_inputs(world, n, local, K)
            for k in range(K):
                buf = data[k][rank].reshape(-1).copy()
                host(desc, buf, local)
                want = mc.pipelined_expected(world, n, data[k], local)[rank]
                bad = int((buf.reshape(local, n) != want[None, :]).sum())
                if bad:
                    fails.append(("pipelined", k, bad))
        else:   # test_config4_one_gib_over_rccl_across_gpus at 1 MiB per rank (auto channels: every link)
            n = 1 << 19
            desc = t.dist_desc(t.SWING, t.BO, side, total, n)
            b = mc.config4_ints(n, rank, "cpu").view(torch.int16).numpy().view(np.uint16).copy()
            host(desc, b, 1)
            got = torch.from_numpy(b.view(np.int16)).view(torch.bfloat16).float()
            bad = int((got != mc.config4_exact(n, world, "cpu")).sum())
            if bad:
                fails.append(("config4", bad))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, fails))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, [("exception", repr(e), traceback.format_exc())]))


@pytest.mark.parametrize("which", ["programs", "pipelined", "config4"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_multidevice_cases_over_the_host_twin(world, which):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q, which)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, fails in results:
        assert fails == [], (rank, fails)
