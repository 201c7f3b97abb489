# round-6: the peer hand-offs under launch skew (random spins ahead of every call) — the hierarchical forms and the
# flat programs, 2 / 4 / 8 processes sharing the GPU, and the multi-device twins rehearsed on device 0
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${R06G_OUT:-r06g}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_peer.py -k skew -v --timeout 300 --timeout-method thread \
    > $out/tests.log 2>&1 &&
ALLRED_TEST_REHEARSE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_multidevice.py -k skew -v --timeout 300 \
    --timeout-method thread > $out/tests_rehearse.log 2>&1
rc=$?
tail -5 $out/tests.log; tail -5 $out/tests_rehearse.log
exit $rc
