# round-3: k_hier_x / k_hier_x2 row stores one tile behind (hier_x_lag) — parity, then A/B (tools/hier_step.py, W = 1)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03j
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_peer.py -x -q -k "pipelined" --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for lag in 0 1; do
  echo "lag=$lag $(ALLRED_TUNE=hier_x_lag=$lag timeout -k 10 150 python tools/hier_step.py 200 3)" >> $out/ab.txt || exit 1
done; done
cat $out/ab.txt
