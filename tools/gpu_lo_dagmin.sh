#!/bin/bash
# GPU session: where the fused LO DAG pipe (lane-group table) starts to pay:
# Swing LO 16..96 kB per rank x 64 ranks, DAG pipe from 1 tile vs the default
# threshold (register butterfly below 256 LDS tiles), arms alternated.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lodagmin}
mkdir -p $OUT
for rep in 1 2 3; do
  for tiles in 8 16 32 48; do
    for m in 1 256; do
      echo -n "DAG_MIN=$m " >> $OUT/ab.txt
      ALLRED_BFLY_DAG_MIN=$m AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py lo $tiles 400 >> $OUT/ab.txt || exit 1
    done
  done
done
echo DONE > $OUT/done
