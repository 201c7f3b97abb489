#!/bin/bash
# GPU session: where the DAG form of the fused LO pays — parity at every LO
# size with the DAG pipe forced from 1 tile (ALLRED_BFLY_DAG_MIN=1), then Swing
# LO 2 kB..640 kB per rank x 64 ranks with the DAG pipe from 1 / 256 LDS tiles /
# never (tools/ab_fused.py, 32 rotating sets, HIP graph replay).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lodag}
mkdir -p $OUT
ALLRED_BFLY_DAG_MIN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lo or LO" -x -q --timeout 100 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for tiles in 1 4 16 32 64 128 256 320; do
  for m in 1 256 1000000; do
    ALLRED_BFLY_DAG_MIN=$m AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py lo $tiles 400 >> $OUT/ab.jsonl || exit 1
  done
done
echo DONE > $OUT/done
