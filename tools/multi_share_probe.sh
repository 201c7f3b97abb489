#!/bin/bash
# Failure rate of the in-process share-device rehearsal (ALLRED_TRANSPORT=peer,
# ALLRED_SHARE_GPU=1) against G, GPU_MAX_HW_QUEUES and the workgroup slots the
# groups' grids divide (ALLRED_SHARE_SLOTS): each run is one CLI process; prints
# "G Q slots rc milliseconds" per run.
out=${1:-gpurun_out/multi_share_probe.txt}
for G in 4 8; do
  for S in ${SLOTS:-512 256 128}; do
    for Q in ${QUEUES:-8 16 32}; do
      for i in 1 2 3 4 5; do
        t0=$(date +%s%3N)
        timeout -k 5 60 env ALLRED_TRANSPORT=peer ALLRED_SHARE_GPU=1 ALLRED_GPUS=$G ALLRED_NODES=$G GPU_MAX_HW_QUEUES=$Q \
          ALLRED_SHARE_SLOTS=$S tenstorrentallreduce_amd/bin/allred_mem_2D 1 1 $([ $G = 8 ] && echo 4 || echo 2) 13 40 32 \
          > /dev/null 2>&1
        rc=$?
        t1=$(date +%s%3N)
        echo "$G $Q $S $rc $((t1 - t0))ms" >> $out
        [ $rc -ge 124 ] && exit $rc
      done
    done
  done
done
exit 0
