# round-3: the schedule form reduced to k_steps_reg (k_steps_pipe / k_steps_wave removed) — parity of every test that
# runs the schedule form, then its default timing at config 2 (BO) and 640 kB (LO)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03w
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_cli.py tests/test_gpu_parity.py -x -q \
    --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for v in "bo 5" "lo 320"; do
  AB_EXEC=steps AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py $v 200 >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done; done
python - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r03w/ab.jsonl"):
    d = json.loads(l); by[(d["variant"], d["bytes_per_rank"])].append(d["us"])
for k, v in sorted(by.items()): print(k, v)
PY
