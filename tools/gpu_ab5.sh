#!/bin/bash
# GPU session: A/B of fused-pass forms.  ARMS = ';'-separated env assignments,
# e.g. ARMS="ALLRED_PIPE_REL=1;ALLRED_PIPE_REL=1 ALLRED_PIPE_CONTIG=1".
# Parity subset per arm, then three interleaved timing rounds.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
IFS=';' read -ra A <<< "$ARMS"
i=0
for arm in "${A[@]}"; do
  i=$((i+1))
  env $arm timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "config2 or fused or config4 or padded or linearity" > $OUT/pytest_arm$i.log 2>&1 || exit 0
done
for r in 1 2 3; do for arm in "${A[@]}"; do
  env $arm AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py ${VARIANT:-bo} ${TILES:-5} 400 >> $OUT/ab.jsonl || exit 0
done; done
echo DONE > $OUT/done
