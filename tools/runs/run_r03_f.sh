# round-3: k_tree_bcast_x balanced-waves A/B, k_broadcast-in-launch-form probe (rocprofv3),
# and this round's rocprofv3 stats + PMC of the N = 1 bench (tools/gpu.sh prof)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03f
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -2 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for bal in 0 1; do ALLRED_TUNE=tree_bcast_bal=$bal timeout -k 10 120 python tools/hier_local.py 200 >> $out/local.jsonl 2>> $out/local.err || exit 1; done; done
python - <<'PY'
import json
for l in open("gpurun_out/r03f/local.jsonl"):
    d = json.loads(l); print(d["env"], d["local_phases"]["tree_bcast_x"]["us"])
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/bp -o run -- python3 tools/bcast_probe.py 100 > $out/bp.out 2> $out/bp.err || exit 1
bash tools/gpu.sh prof r03prof_bench
timeout -k 10 120 python tools/streams_probe.py 100 5 > $out/streams.json 2> $out/streams.err && cat $out/streams.json
