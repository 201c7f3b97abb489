# round-5: k_hier_ws with quarter / half / whole tiles per reducing wave (128 / 256 / 512-byte row segments, 8 / 4 / 2 waves per
# workgroup) against quarter tiles — parity (W = 1, 2 / 4 / 8 processes), W = 1 step times
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05i
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_peer.py \
    -k "hier_forms_single or one_shot_multi_process" > $out/tests.log 2>&1 &&
HIER_ARMS=hier_ll,hier_ws,hier_ws_c16,hier_ws_c16_a2,hier_ws_c32,hier_ws_c32_a2,hier_x2_tail2_lp \
    timeout -k 10 300 python tools/hier_step.py 100 3 > $out/hier_step.json 2> $out/hier_step.err
rc=$?
tail -3 $out/tests.log
python3 -c "import json; d=json.load(open('$out/hier_step.json')); print(d['us_per_step'], d['peer_status'])"
exit $rc
