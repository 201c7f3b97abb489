# round-5: host-staged DMA — default (8 chunks where the box's 2D copies keep the 1D rate, probed) vs
# forced 8 chunks vs one copy each way; then the CLI parity tests of the DMA path
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05k
mkdir -p $out
timeout -k 10 300 python tools/e2e_probe.py 5 > $out/e2e.json 2> $out/e2e.err &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cli.py -k "dma or end_to_end" \
    > $out/tests.log 2>&1
rc=$?
cat $out/e2e.json
tail -2 $out/tests.log
exit $rc
