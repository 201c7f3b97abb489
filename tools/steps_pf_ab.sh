#!/bin/bash
# A/B of the schedule form at config 2: BO (5 tiles) and LO (640 kB) with the
# program words read per phase (steps_prefetch=0) or prefetched (1), and BO with
# two strips per wave body (steps_ilp=2); arms interleaved, 3 rounds each.
out=${1:-gpurun_out/steps_pf_ab.txt}
for r in 1 2 3; do
  for arm in "bo 5|steps_prefetch=0" "bo 5|steps_prefetch=1" "bo 5|steps_ilp=2" "lo 320|steps_prefetch=0" "lo 320|steps_prefetch=1"; do
    v=${arm%%|*}; tn=${arm##*|}
    ALLRED_TUNE=$tn AB_EXEC=steps AB_SETS=32 timeout -k 5 120 python tools/ab_fused.py $v 200 >> $out || exit $?
  done
done
