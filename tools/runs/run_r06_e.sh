# round-6: the whole GPU suite on the final build (resident-limited grids), smoke, the driver's N = 1 invocation,
# its rocprofv3 kernel stats, and the 8-process N > 1 rehearsal under the budget
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${R06E_OUT:-r06e}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --maxfail=5 --timeout 400 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err &&
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$out/prof_bench.json \
    2> $GRAFT_REPO_ROOT/$out/prof.err) &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29561 bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > $out/share_n8.json 2> $out/share_n8.err
rc=$?
tail -2 $out/smoke.log
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['hierarchical_step_w1']['k_hier_ws']['us_per_step'])"
exit $rc
