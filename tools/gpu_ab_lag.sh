#!/bin/bash
# GPU session: the new persistent-kernel parity tests, then A/B of the lagged-store
# fused forms against the round-1 forms (ALLRED_PIPE_LAG=0) for BO, LO and MEM at
# config-2 size, three interleaved rounds, 32 rotating sets (tools/ab_fused.py).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ablag}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "persistent or config2 or lo_sizes" -x -q --timeout 100 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest.log
[ $rc -eq 0 ] || exit 0
for i in 1 2 3; do
  for v in bo lo mem; do
    AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py $v 5 400 >> $OUT/ab.jsonl || exit 0
    ALLRED_PIPE_LAG=0 AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py $v 5 400 >> $OUT/ab.jsonl || exit 0
  done
done
echo DONE > $OUT/done
