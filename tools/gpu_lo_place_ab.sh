#!/bin/bash
# GPU session: fused Swing LO at 128 / 256 / 640 kB x 64 ranks, this build
# (placed DAG, ALLRED_DAG_PLACE=1 / 0) vs the previous build
# (tenstorrentallreduce_amd/build/old/liballred.so), arms alternated.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-loplaceab}
mkdir -p $OUT
OLD=tenstorrentallreduce_amd/build/old/liballred.so
ALLRED_BFLY_DAG_MIN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lo or LO" -x -q --timeout 100 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for tiles in 64 128 320; do
    for arm in new1 new0 old; do
      lib=""; pl=1
      [ $arm = old ] && lib=$OLD
      [ $arm = new0 ] && pl=0
      echo -n "$arm " >> $OUT/ab.txt
      ALLRED_LIB_PATH=$lib ALLRED_DAG_PLACE=$pl AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py lo $tiles 400 >> $OUT/ab.txt || exit 1
    done
  done
done
echo DONE > $OUT/done
