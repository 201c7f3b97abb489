#!/bin/bash
# GPU session: mem_2D schedule form (k_mem<false> + k_broadcast): loads in flight
# per thread (ALLRED_MEM_BATCH) x workgroup size (ALLRED_MEM_BLOCK) arms, after
# mem parity under the two most different arms; 64 ranks, 128 / 256 / 640 kB.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-membatch}
mkdir -p $OUT
for arm in "32 64" "16 128"; do
  set -- $arm
  ALLRED_MEM_BATCH=$1 ALLRED_MEM_BLOCK=$2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -k "mem or MEM" -x -q --timeout 100 --timeout-method thread > $OUT/pytest_$1_$2.log 2>&1
  rc=$?
  echo "PYTEST_EXIT $rc" >> $OUT/pytest_$1_$2.log
  [ $rc -eq 0 ] || exit 1
done
for rep in 1 2; do
  for tiles in 5 1 2; do
    for arm in "8 256" "16 256" "16 64" "32 64" "32 128"; do
      set -- $arm
      echo -n "B=$1 blk=$2 " >> $OUT/ab.txt
      ALLRED_MEM_BATCH=$1 ALLRED_MEM_BLOCK=$2 AB_EXEC=steps AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py mem $tiles 200 >> $OUT/ab.txt || exit 1
    done
  done
done
echo DONE > $OUT/done
