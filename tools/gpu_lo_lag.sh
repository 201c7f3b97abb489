#!/bin/bash
# GPU session (historical: the EX = 5 arm is removed): the fused LO DAG pass with loads two tiles ahead (EX = 5, the
# arm) vs one tile ahead (EX = 4, the default): LO parity with the DAG pipe forced from
# 1 tile, then Swing LO 128 kB..640 kB x 64 ranks, arms alternated.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lolag}
mkdir -p $OUT
ALLRED_BFLY_DAG_MIN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lo or LO" -x -q --timeout 100 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for tiles in 64 128 320; do
    for ex in 5 4; do
      echo -n "EX=$ex " >> $OUT/ab.txt
      ALLRED_BFLY_EX=$ex AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py lo $tiles 400 >> $OUT/ab.txt || exit 1
    done
  done
done
echo DONE > $OUT/done
