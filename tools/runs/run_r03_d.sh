# round-3: k_tree_bcast_x lag 0 / 1 A/B (tools/hier_local.py, interleaved), tests, force-dist bench
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03d
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?; tail -3 $out/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for lag in 0 1; do ALLRED_TUNE=tree_bcast_lag=$lag timeout -k 10 120 python tools/hier_local.py 200 >> $out/local.jsonl 2>> $out/local.err || exit 1; done; done
python - <<'PY'
import json
for l in open("gpurun_out/r03d/local.jsonl"):
    d = json.loads(l); print(d["env"], {k: v["us"] for k, v in d["local_phases"].items()})
PY
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 > $out/fd.json 2> $out/fd.err; rc=$?
tail -2 $out/fd.err
exit $rc
