#!/bin/bash
# GPU session: parity suite + A/B of the early-release pipelined tree forms
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit 0
for i in 1 2 3; do for R in 0 1; do
  ALLRED_PIPE_REL=$R AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py bo 5 400 >> $OUT/ab.jsonl || exit 0
  ALLRED_PIPE_REL=$R AB_SETS=32 timeout -k 10 120 python tools/hier_local.py >> $OUT/hier.jsonl || exit 0
done; done
echo DONE > $OUT/done
