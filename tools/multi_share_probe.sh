#!/bin/bash
# Failure rate of the in-process share-device rehearsal (ALLRED_TRANSPORT=peer,
# ALLRED_SHARE_GPU=1) against GPU_MAX_HW_QUEUES and G: each run is one CLI
# process; prints "G Q rc seconds" per run.
out=${1:-gpurun_out/multi_share_probe.txt}
for G in 4 8; do
  for Q in 4 8 16 32; do
    for i in 1 2 3 4 5; do
      t0=$(date +%s%3N)
      timeout -k 5 60 env ALLRED_TRANSPORT=peer ALLRED_SHARE_GPU=1 ALLRED_GPUS=$G ALLRED_NODES=$G GPU_MAX_HW_QUEUES=$Q \
        tenstorrentallreduce_amd/bin/allred_mem_2D 1 1 $([ $G = 8 ] && echo 4 || echo 2) 13 40 32 > /dev/null 2>&1
      rc=$?
      t1=$(date +%s%3N)
      echo "$G $Q $rc $((t1 - t0))ms" >> $out
      [ $rc -ge 124 ] && exit $rc
    done
  done
done
exit 0
