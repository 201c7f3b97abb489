# round-4: schedule-form A/B across libraries, arms interleaved on one box (config 2, BO 5 tiles / LO 320):
# now = this build; k03 = this build with round 3's kernels.hip; r03 = the round-3 library (cc8d386)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04o
mkdir -p $out
rm -f $out/ab.jsonl
for rep in 1 2 3; do
  for v in "bo 5" "lo 320"; do
    for lib in now k03 r03; do
      ALLRED_LIB_PATH=$PWD/ab_libs/$lib/liballred.so AB_EXEC=steps AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py $v 200 \
        >> $out/ab.jsonl 2>> $out/err || exit 1
    done
    ALLRED_LIB_PATH=$PWD/ab_libs/now/liballred.so ALLRED_TUNE=steps_early=0 AB_EXEC=steps AB_SETS=32 timeout -k 10 120 \
      python tools/ab_fused.py $v 200 >> $out/ab.jsonl 2>> $out/err || exit 1
  done
done
python3 - <<'PY'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/r04o/ab.jsonl"):
    r = json.loads(l)
    by[(r["variant"], r["lib"].split("/")[-2], r["env"].get("ALLRED_TUNE", ""))].append(r["us"])
for k, v in sorted(by.items()):
    print(k, sorted(v))
PY
