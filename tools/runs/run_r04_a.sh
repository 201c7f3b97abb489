# round-4: peer tests (chunked hier_x / x2, flag hand-offs);
# hierarchical step timing at W = 1 with kernel trace + PMC traffic of every form; in-process
# share-device rehearsal of the multi-GPU CLI (probe + tests)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04a
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_peer.py -m gpu > $out/peer.log 2>&1; rc=$?; tail -3 $out/peer.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/hier_step.py 100 3 > $out/hier_step.json 2> $out/hier_step.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- python3 tools/hier_step.py 100 2 > /dev/null 2> $out/tr.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- python3 tools/hier_step.py 20 1 > /dev/null 2> $out/f.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- python3 tools/hier_step.py 20 1 > /dev/null 2> $out/w.err || exit 1
tools/multi_share_probe.sh $out/multi_share_probe.txt || exit 1
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py -m gpu > $out/multi.log 2>&1; rc=$?; tail -3 $out/multi.log
exit $rc
