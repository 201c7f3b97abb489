#!/bin/bash
# GPU session: parity (whole test_gpu_parity.py), then A/B of the fused LO
# routes (ALLRED_LO_TREE=1: rank-uniform schedules run the BO tree pass; 0: the
# butterfly) for RecDub at 640 kB x 64 ranks and for config 1 (2x2, 1 tile).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lotree}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for lt in 1 0; do
    ALLRED_LO_TREE=$lt AB_ALGO=recdub AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py lo 320 400 >> $OUT/ab.jsonl || exit 1
    ALLRED_LO_TREE=$lt AB_ALGO=recdub AB_P=4 AB_SIDE=2 AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py lo 1 2000 >> $OUT/ab.jsonl || exit 1
  done
done
echo DONE > $OUT/done
