# round-5: the whole GPU suite on the round's code (dense hand-offs, fences, chunked DMA, pruned forms),
# then the N > 1 bench rehearsed with 8 processes on the one GPU (candidates, fenced twins, dropped list)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05d
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --maxfail=5 --timeout 400 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?
tail -12 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > $out/share_n8.json 2> $out/share_n8.err
rc=$?
tail -3 $out/share_n8.err
exit $rc
