# round-5: rocprofv3 kernel stats and PMC traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of
# k_hier_ws<1, 16> (the default: half tiles per reducing wave) at W = 1
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05j
mkdir -p $out
HIER_ARMS=hier_ws timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- \
    python3 tools/hier_step.py 100 2 > $out/step.json 2> $out/tr.err &&
HIER_ARMS=hier_ws timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/f.err &&
HIER_ARMS=hier_ws timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/w.err
rc=$?
cat $out/step.json
exit $rc
