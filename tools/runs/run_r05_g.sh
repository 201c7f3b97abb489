# round-5: k_hier_ws — loads one / two tiles ahead, grid caps (3 / 4 tiles per workgroup), then
# rocprofv3 kernel stats and PMC traffic (FETCH_SIZE, WRITE_SIZE in separate passes) at W = 1
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05g
mkdir -p $out
HIER_ARMS=hier_ll,hier_ws,hier_ws_a2,hier_x2_tail2_lp \
    timeout -k 10 300 python tools/hier_step.py 100 3 > $out/hier_step.json 2> $out/hier_step.err &&
HIER_CAP=427 HIER_ARMS=hier_ws,hier_ws_a2 timeout -k 10 200 python tools/hier_step.py 100 3 > $out/cap427.json 2> $out/cap427.err &&
HIER_CAP=320 HIER_ARMS=hier_ws,hier_ws_a2 timeout -k 10 200 python tools/hier_step.py 100 3 > $out/cap320.json 2> $out/cap320.err &&
HIER_ARMS=hier_ws timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- \
    python3 tools/hier_step.py 100 2 > /dev/null 2> $out/tr.err &&
HIER_ARMS=hier_ws timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/f.err &&
HIER_ARMS=hier_ws timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- \
    python3 tools/hier_step.py 20 1 > /dev/null 2> $out/w.err
rc=$?
for f in hier_step cap427 cap320; do
  python3 -c "import json; d=json.load(open('$out/$f.json')); print('$f', d['us_per_step'], d['peer_status'])"
done
exit $rc
