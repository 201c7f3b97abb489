# round-4: k_hier_x2 with old.s results polled in A(cur 0) ahead of its partial push (hier_x_latepoll), TAIL 1 / 2:
# peer tests, then W = 1 step A/B, twice
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04y
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_peer.py -m gpu > $out/peer.log 2>&1; rc=$?; tail -3 $out/peer.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  HIER_ARMS=hier_x_lp,hier_x_re_lp,hier_x2_tail2,hier_x2_tail2_lp,hier_x2_tail_lp timeout -k 10 150 \
    python tools/hier_step.py 200 3 >> $out/hier_x2lp_ab.json 2>> $out/hier_step.err || exit 1
done
python3 -c "
import json
for l in open('$out/hier_x2lp_ab.json'): print(json.loads(l)['us_per_step'])"
