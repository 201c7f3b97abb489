#!/bin/bash
# GPU session: the mem_2D schedule form's reduce as the LDS-staged pass
# (k_mem_lds<P> writing the block sums only) vs k_mem<false, 16>
# (ALLRED_MEM_REDUCE_LDS=0): mem parity under both, A/B at 128 / 256 / 640 kB,
# then a kernel trace of the schedule form at 640 kB.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-memred}
mkdir -p $OUT
for v in 1 0; do
  ALLRED_MEM_REDUCE_LDS=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -k "mem or MEM" -x -q --timeout 100 --timeout-method thread > $OUT/pytest_$v.log 2>&1
  rc=$?
  echo "PYTEST_EXIT $rc" >> $OUT/pytest_$v.log
  [ $rc -eq 0 ] || exit 1
done
for rep in 1 2 3; do
  for tiles in 5 1 2; do
    for v in 1 0; do
      echo -n "LDS=$v " >> $OUT/ab.txt
      ALLRED_MEM_REDUCE_LDS=$v AB_EXEC=steps AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py mem $tiles 200 >> $OUT/ab.txt || exit 1
    done
  done
done
AB_EXEC=steps AB_SETS=32 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o mem --output-format csv -- python3 tools/ab_fused.py mem 5 200 > $OUT/prof.log 2>&1 || exit 1
echo DONE > $OUT/done
