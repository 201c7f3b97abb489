#!/bin/bash
# GPU session: A/B timings (TAG names the output dir; PYTEST=1 runs the parity suite first,
# with the A/B env of PYTEST_ENV).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
if [ -n "$PYTEST" ]; then
  env $PYTEST_ENV timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "PYTEST_EXIT $rc" >> $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit 0
fi
for i in 1 2 3; do
  AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py bo 5 400 >> $OUT/ab.jsonl || exit 0
  ALLRED_PIPE_REL=1 AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py bo 5 400 >> $OUT/ab.jsonl || exit 0
done
echo DONE > $OUT/done
