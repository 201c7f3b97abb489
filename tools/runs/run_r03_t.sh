# round-3: k_steps_reg grid — every wave at least 1 (default) or 2 strips (tune steps_reg_spw) at 512 and 640 kB per rank
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03t
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -k "schedule_form" \
    --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for spw in 1 2; do for v in "bo 5" "bo 4" "lo 320" "lo 256"; do
  AB_EXEC=steps AB_SETS=32 ALLRED_TUNE=steps_reg_spw=$spw timeout -k 10 120 python tools/ab_fused.py $v 200 >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done; done; done
python - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r03t/ab.jsonl"):
    d = json.loads(l); by[(d["variant"], d["bytes_per_rank"], d["env"].get("ALLRED_TUNE"))].append(d["us"])
for k, v in sorted(by.items()): print(k, v)
PY
