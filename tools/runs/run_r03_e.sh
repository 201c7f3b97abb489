# round-3: full GPU suite + smoke, then k_tree_bcast_x<1> rocprofv3 stats and PMC
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03e
mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -rf --maxfail=10 --timeout 240 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -8 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- python3 tools/hier_local.py 200 > $out/local.json 2> $out/tr.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- python3 tools/hier_local.py 50 > /dev/null 2> $out/f.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- python3 tools/hier_local.py 50 > /dev/null 2> $out/w.err || exit 1
cat $out/local.json
