# round-6: the whole multi-device suite rehearsed on one GPU at HEAD (ALLRED_TEST_REHEARSE=1: the peer-window
# cases with every rank on device 0; the RCCL cases skip — RCCL refuses two ranks on one device)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${R06Q_OUT:-r06q}
mkdir -p $out
ALLRED_TEST_REHEARSE=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_multidevice.py -m gpu -q -rs \
    --maxfail=5 --timeout 400 --timeout-method thread > $out/tests.log 2>&1
rc=$?
tail -12 $out/tests.log
exit $rc
