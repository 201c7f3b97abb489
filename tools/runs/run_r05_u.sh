# round-5: the fused BO pass over half tiles (k_tree_lds_lag<64, 16>: 256-byte rank-row segments, twice the
# tiles per workgroup, a quarter of the LDS) — parity with ALLRED_TUNE=fused_tv=16, then config-2 step times
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05u
mkdir -p $out
ALLRED_TUNE=fused_tv=16 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_configs.py -k "fused or FUSED or config2 or parity" > $out/tests.log 2>&1
rc=$?
tail -2 $out/tests.log
[ $rc -eq 0 ] || exit $rc
export AB_EAGER=1 AB_SETS=32
for r in 1 2 3; do
  for tn in "fused_tv=32" "fused_tv=16" "fused_tv=16,pipe_grid=768" "fused_tv=16,pipe_grid=1024"; do
    ALLRED_TUNE=$tn timeout -k 10 120 python tools/ab_fused.py bo 5 200 > $out/ab.json 2> $out/ab.err || exit 1
    python3 -c "import json; d=json.load(open('$out/ab.json')); print('$tn', d['us'])"
  done
done
