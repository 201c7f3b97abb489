# round-5: the 64-rank LO schedule form with a loader wave + four chain waves (k_steps_lo_split) against
# k_steps_reg — parity, then config-2 step times (tools/ab_fused.py, arms interleaved)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05p
mkdir -p $out
export AB_EAGER=1 AB_SETS=32 AB_EXEC=steps
for r in 1 2; do
  for tn in "steps_lo_split=0" "steps_lo_split=1,pipe_grid=512" "steps_lo_split=1,pipe_grid=384" "steps_lo_split=1,pipe_grid=256" "steps_lo_split=2,pipe_grid=512" "steps_lo_split=2,pipe_grid=384"; do
    ALLRED_TUNE=$tn timeout -k 10 120 python tools/ab_fused.py lo 320 200 > $out/ab.json 2> $out/ab.err || exit 1
    python3 -c "import json; d=json.load(open('$out/ab.json')); print('$tn', d['us'])"
  done
done
