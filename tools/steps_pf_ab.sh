#!/bin/bash
# A/B of the schedule form's program-word prefetch (tune steps_prefetch) at
# config 2: BO (5 tiles) and LO (640 kB), arms interleaved, 3 rounds each.
out=${1:-gpurun_out/steps_pf_ab.txt}
for r in 1 2 3; do
  for v in "bo 5" "lo 320"; do
    for pf in 0 1; do
      ALLRED_TUNE=steps_prefetch=$pf AB_EXEC=steps AB_SETS=32 timeout -k 5 120 python tools/ab_fused.py $v 200 >> $out || exit $?
    done
  done
done
