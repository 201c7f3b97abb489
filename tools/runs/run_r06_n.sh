# round-6: the peer GPU tests as committed (skew, epoch-wrap with a late process) and the multi-device twins of the
# new cases rehearsed with every rank on device 0
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06n
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_peer.py -q -rs --timeout 300 --timeout-method thread \
    > $out/peer.log 2>&1 &&
ALLRED_TEST_REHEARSE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_multidevice.py -k "wrap or skew" -q \
    --timeout 300 --timeout-method thread > $out/rehearse.log 2>&1
rc=$?
tail -3 $out/peer.log; tail -3 $out/rehearse.log
exit $rc
