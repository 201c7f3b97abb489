# round-4: the schedule form of this build vs the round-3 library (ab_libs/r03, built from commit cc8d386)
# in one process order, arms interleaved, config 2 BO (5 tiles) and LO (320), 32 rotating sets, graph replays
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04n
mkdir -p $out
for rep in 1 2 3; do
  for v in "bo 5" "lo 320"; do
    AB_EXEC=steps AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py $v 200 >> $out/ab.jsonl 2>> $out/err || exit 1
    AB_EXEC=steps AB_SETS=32 ALLRED_TUNE=steps_early=0 timeout -k 10 120 python tools/ab_fused.py $v 200 >> $out/ab.jsonl 2>> $out/err || exit 1
    ALLRED_LIB_PATH=$PWD/ab_libs/r03/liballred.so AB_EXEC=steps AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py $v 200 \
      >> $out/ab.jsonl 2>> $out/err || exit 1
  done
done
python3 - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r04n/ab.jsonl"):
    r = json.loads(l)
    by[(r["variant"], "r03" if r["lib"] else "r04", r["env"].get("ALLRED_TUNE", ""))].append(r["us"])
for k, v in sorted(by.items()):
    print(k, sorted(v))
PY
