# round-5: the whole GPU suite on the round's code (dense hand-offs, fences, chunked DMA, pruned forms,
# LO schedule form storing from registers), rocprofv3 of the schedule forms (BO / LO, config 2 size),
# then the N > 1 bench rehearsed with 8 processes on the one GPU (candidates, fenced twins, dropped list)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05d
mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rs --maxfail=5 --timeout 400 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?
tail -12 $out/tests.log
[ $rc -eq 0 ] || exit $rc
export AB_EAGER=1 AB_SETS=32
AB_EXEC=steps timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $out/steps_bo -o run -- \
    python3 tools/ab_fused.py bo 5 200 > $out/steps_bo.json 2> $out/e3 &&
AB_EXEC=steps timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $out/steps_lo -o run -- \
    python3 tools/ab_fused.py lo 320 200 > $out/steps_lo.json 2> $out/e4 &&
cat $out/steps_bo.json $out/steps_lo.json &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > $out/share_n8.json 2> $out/share_n8.err
rc=$?
tail -3 $out/share_n8.err
exit $rc
