rm -f gpurun_out/pad.jsonl
for rep in 1 2; do
for pad in 0 64 128 256 512 1024 2048 4096 192; do
  AB_PAD=$pad AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py bo 5 200 >> gpurun_out/pad.jsonl 2>>gpurun_out/pad.err || exit 1
done; done
python - <<'PY'
import json, collections
by=collections.defaultdict(list)
for l in open("gpurun_out/pad.jsonl"):
    r=json.loads(l); by[int(r["env"]["AB_PAD"])].append(r["us"])
for k in sorted(by): print(k*2, "B skew:", sorted(by[k]))
PY
