# round-3: k_steps_reg with one register set (next strip loaded after step 0): 3 / 4 / 5 groups per CU — parity, A/B
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03q
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -k "schedule_form" \
    --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for sw in 5 6 7; do for v in "bo 5" "lo 320"; do
  AB_EXEC=steps AB_SETS=32 ALLRED_TUNE=steps_wave=$sw timeout -k 10 120 python tools/ab_fused.py $v 200 >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done; done; done
python - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r03q/ab.jsonl"):
    d = json.loads(l); by[(d["variant"], d["env"].get("ALLRED_TUNE"))].append(d["us"])
for k, v in sorted(by.items()): print(k, v)
PY
echo "steps_wave=6 $(ALLRED_TUNE=steps_wave=6 timeout -k 10 120 python tools/steps_phases.py bo)" >> $out/phases.txt || exit 1
cat $out/phases.txt
