# round-5: the hierarchical forms with the 7 + 1 byte hand-off words — parity (W = 1 and 2 / 4 / 8
# processes, the epoch-wrap clear), W = 1 step times, rocprofv3 + PMC traffic of the kernels, then
# the N = 1 bench line with the chunked-DMA variants
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05c
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_peer.py -m gpu -q -rs -x --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1
rc=$?
tail -8 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/hier_step.py 100 3 > $out/hier_step.json 2> $out/hier_step.err && cat $out/hier_step.json && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- python3 tools/hier_step.py 100 2 > /dev/null 2> $out/tr.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- python3 tools/hier_step.py 20 1 > /dev/null 2> $out/f.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- python3 tools/hier_step.py 20 1 > /dev/null 2> $out/w.err && \
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?
tail -3 $out/bench.err
python -c "import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['roofline']['frac'], json.dumps(d['host_staged']))"
exit $rc
