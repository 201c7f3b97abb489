# round-5: the multi-device suite rehearsed on one GPU (peer cases, every rank on device 0), the peer
# tests with the fenced forms, the N > 1 bench rehearsal (fenced twins, dropped list), W = 1 hier step timing
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05a
mkdir -p $out
ALLRED_TEST_REHEARSE=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_multidevice.py tests/test_gpu_peer.py tests/test_abi.py \
    -m gpu -q -rs -x --timeout 400 --timeout-method thread > $out/tests.log 2>&1
rc=$?
tail -30 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/hier_step.py 100 3 > $out/hier_step.json 2> $out/hier_step.err && cat $out/hier_step.json && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --share-gpu --steps 20 --warmup 5 > $out/share_n2.json 2> $out/share_n2.err
rc=$?
tail -5 $out/share_n2.err
exit $rc
