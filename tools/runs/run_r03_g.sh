set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03g
mkdir -p $out
for r in 1 2; do NO_PEER=1 timeout -k 10 120 python tools/bcast_probe.py 200 >> $out/bp_ev2.out 2>> $out/bp_ev2.err || exit 1; done; cat $out/bp_ev2.out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_peer.py -x -q --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 > $out/fd.json 2> $out/fd.err; rc=$?; tail -1 $out/fd.err
python - <<'PY'
import json
d = json.load(open("gpurun_out/r03g/fd.json")); x = d["xgmi"]
print(d["config"]["transport"], d["ms_per_step"], x["transport_quick_ms"], x["local_phases_ms"])
PY
exit $rc
