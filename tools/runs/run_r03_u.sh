# round-3: k_steps_reg grid, steps_reg_spw 1 vs 2 over the reference's BO / LO size sweep (128-640 kB per rank)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03u
mkdir -p $out
for r in 1 2 3; do for spw in 1 2; do for v in "bo 1" "bo 2" "bo 3" "lo 64" "lo 128" "lo 192"; do
  AB_EXEC=steps AB_SETS=32 ALLRED_TUNE=steps_reg_spw=$spw timeout -k 10 120 python tools/ab_fused.py $v 200 >> $out/ab.jsonl 2>> $out/ab.err || exit 1
done; done; done
python - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r03u/ab.jsonl"):
    d = json.loads(l); by[(d["variant"], d["bytes_per_rank"], d["env"].get("ALLRED_TUNE"))].append(d["us"])
for k, v in sorted(by.items()): print(k, v)
PY
