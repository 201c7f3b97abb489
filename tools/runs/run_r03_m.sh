# round-3: k_steps_wave with 2 / 3 / 4 strip buffers per wave; k_hier_x / k_hier_x2<TAIL> with the result
# polls ahead of the first tiles' loads — parity, then A/B (tools/ab_fused.py AB_EXEC=steps; tools/hier_step.py)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03m
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_peer.py -x -q -k "schedule_form or peer" \
    --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for sw in 0 1 2 3 4; do for v in "bo 5" "lo 320"; do
  AB_EXEC=steps AB_SETS=32 ALLRED_TUNE=steps_wave=$sw timeout -k 10 120 python tools/ab_fused.py $v 200 >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done; done; done
python - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r03m/ab.jsonl"):
    d = json.loads(l); by[(d["variant"], d["env"].get("ALLRED_TUNE"))].append(d["us"])
for k, v in sorted(by.items()): print(k, v)
PY
for r in 1 2; do
  timeout -k 10 150 python tools/hier_step.py 200 3 >> $out/hier.jsonl 2>> $out/hier.err || exit 1
done
cat $out/hier.jsonl
