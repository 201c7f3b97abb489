#!/bin/bash
# GPU session: the schedule (steps) form's per-step kernel, k_step (one thread
# per 16-byte vector, grid x covers a block) vs k_step_w (one wave per rank
# block, 8 vectors' loads in flight per lane; ALLRED_STEP_FORM=1): parity of
# the step-form tests under the new form, BO / LO steps A/B, per-step trace.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-stepform}
mkdir -p $OUT
ALLRED_STEP_FORM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py -x -q --timeout 100 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for tiles in 5 2 1; do
    for f in 1 0; do
      echo -n "FORM=$f " >> $OUT/ab.txt
      ALLRED_STEP_FORM=$f AB_EXEC=steps AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py bo $tiles 100 >> $OUT/ab.txt || exit 1
    done
  done
done
ALLRED_STEP_FORM=1 AB_EXEC=steps AB_SETS=32 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bo --output-format csv -- python3 tools/ab_fused.py bo 5 100 > $OUT/prof.log 2>&1 || exit 1
echo DONE > $OUT/done
