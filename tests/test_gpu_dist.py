"""The RCCL path on one GPU: a 1-rank communicator (RCCL refuses two ranks on
one device, so N>1 is covered by test_dist_host.py's identical step program
over gloo and by the driver's multi-GPU run).  Checks communicator setup and
the hierarchical stages (on-GPU tree reduce + broadcast) against the host
twin and the oracle, bit for bit."""
import numpy as np
import pytest

import oracle
import tenstorrentallreduce_amd as t

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


# 2,560 elements: one tile per workgroup; 327,680 (config 2, 1,280 tiles) and
# 1,061 tiles (ragged over the 512-workgroup persistent grid): the pipelined form
@pytest.mark.parametrize("n", [64 * 8 * 5, 327680, 1061 * 256])
def test_tree_reduce_and_broadcast_match_oracle(n):
    side, total = 8, 64
    rng = np.random.default_rng(9)
    ranks = [rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(total)]
    buf = torch.from_numpy(np.stack(ranks).view(np.int16)).to(DEV)
    out = torch.empty(n, dtype=torch.int16, device=DEV)
    for algo in (t.SWING, t.RECDUB):
        t.tree_reduce(buf.data_ptr(), n, n, algo, side, total, out.data_ptr())
        torch.cuda.synchronize()
        want = [r.copy() for r in ranks]
        oracle.allreduce("lo", algo, side, want, total)   # LO value of rank 0 = tree of rank 0
        assert np.array_equal(out.cpu().numpy().view(np.uint16), want[0])
    t.broadcast(buf.data_ptr(), n, n, total, out.data_ptr())
    torch.cuda.synchronize()
    got = buf.cpu().numpy().view(np.uint16)
    assert (got == got[0]).all() and np.array_equal(got[0], out.cpu().numpy().view(np.uint16))


@pytest.mark.parametrize("local", [1, 64])
def test_single_rank_rccl_comm(local):
    comm = t.Comm(t.Comm.unique_id(), 1, 0, 0)
    n = 8 * 64 * 4
    rng = np.random.default_rng(local)
    data = [rng.integers(0x3F80, 0x42C8, n).astype(np.uint16) for _ in range(local)]
    buf = torch.from_numpy(np.concatenate(data).view(np.int16)).to(DEV)
    desc = t.dist_desc(t.SWING, t.BO, 1, 1, n, local_ranks=local, local_side=8 if local == 64 else 1,
                       local_algo=t.SWING)
    ws = torch.empty(t.dist_workspace_bytes(desc), dtype=torch.uint8, device=DEV)
    t.dist_allreduce(comm, desc, buf.data_ptr(), ws.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    host = np.concatenate(data).astype(np.uint16)
    scratch = np.zeros(2 * n, dtype=np.uint16)

    def no_exchange(peer, sends, recvs):
        raise AssertionError("a 1-rank grid has no exchange steps")

    t.dist_allreduce_host(desc, 0, host, scratch, no_exchange)
    assert np.array_equal(buf.cpu().numpy().view(np.uint16), host)
    # a bucket or workspace off 16-byte alignment is refused before any exchange
    with pytest.raises(t.AllredError):
        t.dist_allreduce(comm, desc, buf.data_ptr() + 2, ws.data_ptr(), torch.cuda.current_stream())
    with pytest.raises(t.AllredError):
        t.dist_allreduce(comm, desc, buf.data_ptr(), ws.data_ptr() + 8, torch.cuda.current_stream())
    comm.close()
