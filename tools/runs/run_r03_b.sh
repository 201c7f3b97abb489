# round-3 profiling run: k_add (tile-sum) kernel stats + PMC per size, hierarchical kernels' PMC,
# then the N > 1 bench path with a 1-rank RCCL communicator (--force-dist: the RCCL verification)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03prof
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/ts_trace -o run -- \
    python3 bench.py --tilesum-only 256 1024 --steps 50 > $out/ts.json 2> $out/ts.err || exit 1
for mib in 256 1024; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/ts_fetch_$mib -o run -- \
      python3 bench.py --tilesum-only $mib --steps 20 --reps 2 > /dev/null 2> $out/tsf$mib.err || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/ts_write_$mib -o run -- \
      python3 bench.py --tilesum-only $mib --steps 20 --reps 2 > /dev/null 2> $out/tsw$mib.err || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/h_fetch -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/hf.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/h_write -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/hw.err || exit 1
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 > $out/fd.json 2> $out/fd.err; rc=$?
tail -3 $out/fd.err; head -c 600 $out/fd.json
find $out -name "*.csv" | head -30
exit $rc
