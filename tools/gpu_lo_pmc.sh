#!/bin/bash
# GPU session: SQ counters of the fused LO DAG pass (EX = 4, 5) and the fused BO
# pass at 640 kB x 64 ranks, one rocprofv3 --pmc pass each (8 SQ counters).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lopmc}
mkdir -p $OUT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"
for arm in lo4 lo5 bo; do
  v=${arm:0:2}; ex=${arm:2:1}; tiles=320; [ $v = bo ] && tiles=5
  ALLRED_BFLY_EX=${ex:-4} AB_EAGER=1 AB_SETS=32 timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/$arm -o pmc --output-format csv -- python3 tools/ab_fused.py $v $tiles 100 > $OUT/$arm.log 2>&1 || exit 1
done
echo DONE > $OUT/done
