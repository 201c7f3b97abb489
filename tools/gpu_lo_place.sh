#!/bin/bash
# GPU session: the fused LO DAG pass with the bank-conflict-free placement of
# its nodes (default) vs first-appearance rows and slots (ALLRED_DAG_PLACE=0):
# LO parity with the DAG pipe forced from 1 tile (both placements), Swing LO
# 128 / 256 / 640 kB x 64 ranks alternated, then SQ_LDS_BANK_CONFLICT per arm.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-loplace}
mkdir -p $OUT
for pl in 1 0; do
  ALLRED_DAG_PLACE=$pl ALLRED_BFLY_DAG_MIN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lo or LO" -x -q --timeout 100 --timeout-method thread > $OUT/pytest_place$pl.log 2>&1
  rc=$?
  echo "PYTEST_EXIT $rc" >> $OUT/pytest_place$pl.log
  [ $rc -eq 0 ] || exit 1
done
for rep in 1 2 3; do
  for tiles in 64 128 320; do
    for pl in 1 0; do
      echo -n "PLACE=$pl " >> $OUT/ab.txt
      ALLRED_DAG_PLACE=$pl AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py lo $tiles 400 >> $OUT/ab.txt || exit 1
    done
  done
done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"
for pl in 1 0; do
  ALLRED_DAG_PLACE=$pl AB_EAGER=1 AB_SETS=32 timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/pmc$pl -o pmc --output-format csv -- python3 tools/ab_fused.py lo 320 100 > $OUT/pmc$pl.log 2>&1 || exit 1
done
echo DONE > $OUT/done
