# round-6: the N > 1 bench's last-resort watchdog (a forced host-side hang before anything is measured, and
# after the headline) and the contract tests of the N > 1 line, then the 2-process rehearsal as the driver
# would run it
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${R06R_OUT:-r06r}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_bench_multi.py -v -rs --timeout 400 --timeout-method thread \
    > $out/tests.log 2>&1 &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29581 bench.py --gpus 2 --share-gpu --steps 20 --warmup 5 > $out/share_n2.json 2> $out/share_n2.err
rc=$?
tail -8 $out/tests.log
exit $rc
