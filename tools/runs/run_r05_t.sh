# round-5: the whole GPU suite on the final build (k_hier_ws the default, per-test bounds, the bench's W = 1 hierarchical step),
# smoke, the N = 1 bench line as the driver runs it, and a rocprofv3 summary of that bench
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05t
mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rs --maxfail=5 --timeout 400 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?
tail -12 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/prof -o run -- \
    python3 bench.py --main-only --steps 200 --warmup 20 > $out/prof_bench.json 2> $out/prof.err
rc=$?
tail -2 $out/smoke.log
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d.get('host_staged'))[:600])"
exit $rc
