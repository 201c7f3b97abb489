#!/bin/bash
# GPU session: the fused LO pass's arms (ALLRED_BFLY_EX: 0 the ds_bpermute
# butterfly, 4 the DAG of distinct sums — the default; arms 1-3 and 5 were
# measured and removed, profiles/r01_lo_exchange_arms.txt): parity of each arm
# on the persistent-form tests, then interleaved A/B at 640 kB (Swing and RecDub,
# RecDub kept off the BO route), 32 rotating sets (tools/ab_fused.py).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abbfly}
mkdir -p $OUT
ARMS=${ARMS:-"4 0"}
for ex in $ARMS; do
  ALLRED_LO_TREE=0 ALLRED_BFLY_EX=$ex timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "persistent or lo_sizes or lds_forms or rank_uniform" -x -q --timeout 100 --timeout-method thread > $OUT/pytest_ex$ex.log 2>&1
  rc=$?
  echo "PYTEST_EXIT $rc" >> $OUT/pytest_ex$ex.log
  [ $rc -eq 0 ] || exit 1
done
for i in 1 2 3; do
  for ex in $ARMS; do
    for algo in swing recdub; do
      ALLRED_LO_TREE=0 AB_ALGO=$algo ALLRED_BFLY_EX=$ex AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py lo 320 400 >> $OUT/ab.jsonl || exit 1
    done
  done
done
echo DONE > $OUT/done
