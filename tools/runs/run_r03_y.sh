# round-3: two tiles in flight in the read-only passes (k_tree_lds_pipe<P, false>, k_hier_ll's A phase) — parity,
# then the hierarchical forms at W = 1 (tools/hier_step.py: launches = tree + exchange + broadcast, hier_ll)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03y
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_dist.py -x -q --timeout 200 \
    --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 150 python tools/hier_step.py 200 3 >> $out/hier.jsonl 2>> $out/hier.err || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r03y/hier.jsonl"):
    d = json.loads(l); print(d["us_per_step"])
PY
