# round-3 check run: new/changed GPU tests, N = 1 bench (tilesum), 2-process shared-GPU rehearsal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_bench_multi.py tests/test_gpu_peer.py::test_hier_pipelined_single_gpu_bit_exact tests/test_gpu_dist.py tests/test_gpu_parity.py::test_fused_chunked_launches_bit_exact -x -v --timeout 240 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -15 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.json 2> gpurun_out/b1.err || { tail -20 gpurun_out/b1.err; exit 1; }
head -c 1500 gpurun_out/b1.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --share-gpu --steps 20 --warmup 5 > gpurun_out/share2.json 2> gpurun_out/share2.err; rc=$?; tail -5 gpurun_out/share2.err; exit $rc
