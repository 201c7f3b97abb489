# round-6: ABI-7 build — the DMA probe / epoch-wrap / peer tests, smoke, PMC traffic of k_hier_ws and k_hier_x2,
# the driver's N = 1 invocation and its rocprofv3 kernel trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06c
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_peer.py -q -rs --maxfail=3 --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1
rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
HIER_ARMS=hier_ws,hier_x2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/f.err &&
HIER_ARMS=hier_ws,hier_x2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/w.err &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err &&
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$out/prof_bench.json \
    2> $GRAFT_REPO_ROOT/$out/prof.err)
rc=$?
tail -2 $out/smoke.log
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
print(json.dumps(d['hierarchical_step_w1'])[:1200])"
exit $rc
