# round-3: k_steps_reg (BO schedule form, strips staged in registers, step 0 as the rows arrive) — parity, then
# A/B against k_steps_pipe (0) and k_steps_wave (2) (tools/ab_fused.py, AB_EXEC=steps, 32 sets), then stamps
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03n
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -k "schedule_form" \
    --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for sw in 0 2 5; do
  AB_EXEC=steps AB_SETS=32 ALLRED_TUNE=steps_wave=$sw timeout -k 10 120 python tools/ab_fused.py bo 5 200 >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done; done
python - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r03n/ab.jsonl"):
    d = json.loads(l); by[(d["variant"], d["env"].get("ALLRED_TUNE"))].append(d["us"])
for k, v in sorted(by.items()): print(k, v)
PY
echo "steps_wave=5 $(ALLRED_TUNE=steps_wave=5 timeout -k 10 120 python tools/steps_phases.py bo)" >> $out/phases.txt || exit 1
cat $out/phases.txt
# fused pass A/B (tools/ubench/fused_ab): 256-byte-row tiles (2560 per launch, 5 per workgroup at grid 512)
timeout -k 10 180 tools/ubench/fused_ab 200 > $out/fused_ab.jsonl 2> $out/fused_ab.err || exit 1
python - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r03n/fused_ab.jsonl"):
    d = json.loads(l)
    if "us" in d: by[d["form"]].append(d["us"])
    else: print(d)
for k, v in by.items(): print(k, v)
PY
