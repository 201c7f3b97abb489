"""Child process of tests/test_gpu_multi.py and tests/test_gpu_multidevice.py:
allred_run across G GPUs on arbitrary per-rank data — the backend from
ALLRED_TRANSPORT (peer, the default here, or rccl) and ALLRED_SHARE_GPU
(every group on ONE device, G threads whose kernels wait for each other; 0:
group g on device g); writes every rank's result to an .npy file for the
parent to compare with the oracle's composition.  A process of its own so that GPU_MAX_HW_QUEUES (set by the
parent, > G + 1: one hardware queue per thread's stream, no two of the
mutually waiting kernels serialised on one queue) holds from HIP's first call.

usage: gpu_multi_child.py <variant> <gpus> <nodes or -> <seed> <out.npy> -- argv..."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import tenstorrentallreduce_amd as t  # noqa: E402
from multi_cases import random_inputs  # noqa: E402


def main():
    variant, g, nodes, seed, out_path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5]
    argv = ["x", *sys.argv[sys.argv.index("--") + 1:]]
    if nodes != "-":
        os.environ["ALLRED_NODES"] = nodes
    plan = t.multi_plan(argv, variant, gpus=g)
    data = random_inputs(plan.total_nodes, int(plan.elems), seed)
    transport = {"peer": t.TRANSPORT_PEER, "rccl": t.TRANSPORT_RCCL}[os.environ.get("ALLRED_TRANSPORT", "peer")]
    share = os.environ.get("ALLRED_SHARE_GPU", "1") not in ("", "0")
    rep, out = t.run_multi(argv, variant, gpus=g, transport=transport, share_device=share, inputs=data)
    np.save(out_path, np.stack([data, out]))
    print(f"ok device_s={rep.device_seconds:.6f}", flush=True)


if __name__ == "__main__":
    main()
