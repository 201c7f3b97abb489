# round-5: the peer / bench GPU tests with k_hier_ws as the library default
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05q
mkdir -p $out
timeout -k 10 800 python -u -m pytest -q -rs --maxfail=3 --timeout 400 --timeout-method thread tests/test_gpu_peer.py \
    tests/test_gpu_bench_multi.py tests/test_gpu_multi.py > $out/tests.log 2>&1
rc=$?
tail -5 $out/tests.log
exit $rc
