# round-6: the driver's N = 1 invocation (bench.py --gpus 1 --steps 20 --warmup 5) with the secondary kernels
# timed like the headline (spin kernel, R repetitions, median, grid / residency), then a rocprofv3 kernel
# trace of exactly that invocation (verdict r05 item 1); the W = 1 hierarchical parity tests first
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06a
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -k "single_gpu" -x -q --timeout 120 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err &&
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$out/prof_bench.json 2> $GRAFT_REPO_ROOT/$out/prof.err)
rc=$?
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
print(json.dumps(d['hierarchical_step_w1'])[:1500])
print(json.dumps(d['schedule_faithful'])[:800])"
exit $rc
