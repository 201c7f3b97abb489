# round-5: k_hier_ws (the hierarchical one-launch step with reducing and writing waves)
# parity at W = 1 and 2 / 4 / 8 processes, then its step time against k_hier_ll and its knobs
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05f
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_peer.py \
    -k "hier_forms_single or one_shot_multi_process or knob" > $out/tests.log 2>&1 &&
HIER_ARMS=hier_ll,hier_ws,hier_x2_tail2_lp \
    timeout -k 10 300 python tools/hier_step.py 100 3 > $out/hier_step.json 2> $out/hier_step.err &&
HIER_ARMS=hier_ll,hier_ws timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- \
    python tools/hier_step.py 50 2 > $out/prof.log 2>&1
rc=$?
tail -3 $out/tests.log
python3 -c "import json; d=json.load(open('$out/hier_step.json')); print(d['median'], d['peer_status'])"
exit $rc
