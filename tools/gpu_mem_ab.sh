#!/bin/bash
# GPU session: mem_2D parity (every test naming mem / MEM / oneshot / persistent),
# then the fused mem_2D pass at 640 kB x 64 ranks (tools/ab_fused.py, 32 sets),
# and at 128 / 256 kB (k_mem_lds one tile per workgroup).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-memab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -k "mem or MEM or persistent or lds_forms or bit_exact" -x -q --timeout 100 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
OLD=tenstorrentallreduce_amd/build/old/liballred.so   # the previous build, if present: A/B
for i in 1 2 3; do
  for lib in "" $( [ -f $OLD ] && echo $OLD ); do
  export ALLRED_LIB_PATH=$lib
  for tiles in 5 1 2; do
    AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py mem $tiles 400 >> $OUT/ab.jsonl || exit 1
    AB_EXEC=steps AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py mem $tiles 200 >> $OUT/ab.jsonl || exit 1
    AB_P=8 AB_SIDE=4 AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py mem $tiles 400 >> $OUT/ab.jsonl || exit 1
  done
  done
done
echo DONE > $OUT/done
