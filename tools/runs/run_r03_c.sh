# round-3: the pipelined RCCL step (k_tree_bcast_x) — tests, local-phase timing, rocprofv3 stats + PMC,
# then the N > 1 bench path with a 1-rank RCCL communicator (--force-dist)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03c
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -12 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 120 python tools/hier_local.py 200 >> $out/local.jsonl 2>> $out/local.err || exit 1; done
cat $out/local.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- python3 tools/hier_local.py 200 > /dev/null 2> $out/tr.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- python3 tools/hier_local.py 50 > /dev/null 2> $out/f.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- python3 tools/hier_local.py 50 > /dev/null 2> $out/w.err || exit 1
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 > $out/fd.json 2> $out/fd.err; rc=$?
tail -3 $out/fd.err; head -c 300 $out/fd.json
exit $rc
