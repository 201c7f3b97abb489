# round-6: the pruned build (ABI 7: k_hier_ll, k_hier_x and their tune keys retired; k_hier_x2 in its
# product form only) — the launch-gap probe (does a live peer set slow other kernels' dispatch?) plain
# and under a kernel trace, the whole GPU suite, smoke, and PMC passes of the two hierarchical kernels
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06b
mkdir -p $out
timeout -k 10 120 python tools/gap_probe.py 50 5 > $out/gap.json 2> $out/gap.err &&
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/$out/gapprof -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/gap_probe.py 50 5 > $GRAFT_REPO_ROOT/$out/gap_prof.json 2> $GRAFT_REPO_ROOT/$out/gap_prof.err)
rc=$?
cat $out/gap.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --maxfail=5 --timeout 400 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?
tail -6 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
HIER_ARMS=hier_ws,hier_x2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/f.err &&
HIER_ARMS=hier_ws,hier_x2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/w.err
rc=$?
tail -2 $out/smoke.log
exit $rc
