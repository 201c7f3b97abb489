#!/bin/bash
# GPU session: grid-size arms of the lagged fused BO pass (ALLRED_PIPE_GRID), config 2,
# 32 rotating sets, interleaved rounds (tools/ab_fused.py).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abgrid}
mkdir -p $OUT
for i in 1 2; do
  for g in ${GRIDS:-384 448 512 576 640 768}; do
    ALLRED_PIPE_GRID=$g AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py bo 5 400 >> $OUT/ab.jsonl || exit 0
  done
done
echo DONE > $OUT/done
