# round-3: k_hier_x2d (k_hier_x2 with the owned sums at the end and old's results LDS-DMA'd per tile) — parity, A/B at W = 1
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03s
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_peer.py -x -q -k "pipelined2" --timeout 200 --timeout-method thread \
    > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 150 python tools/hier_step.py 200 3 >> $out/hier.jsonl 2>> $out/hier.err || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r03s/hier.jsonl"):
    d = json.loads(l); print({k: v for k, v in d["us_per_step"].items()})
PY
