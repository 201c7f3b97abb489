# round-4: the share-device rehearsal with Finish before the read-back (no D2H queued behind a waiting allreduce);
# the groups released after every thread, the status word read on the group's stream; phase trace of every run;
# then the GPU multi tests at G = 2, 4, 8
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04e
mkdir -p $out
export ALLRED_TRANSPORT=peer ALLRED_SHARE_GPU=1 GPU_MAX_HW_QUEUES=16 ALLRED_MULTI_TRACE=1
for G in 4 8; do
  for i in 1 2 3 4 5 6 7 8; do
    t0=$(date +%s%3N)
    timeout -k 5 60 env ALLRED_GPUS=$G ALLRED_NODES=$G tenstorrentallreduce_amd/bin/allred_mem_2D 1 1 $([ $G = 8 ] && echo 4 || echo 2) 13 40 32 \
      > $out/g$G.run$i.out 2> $out/g$G.run$i.err
    rc=$?
    echo "G=$G run$i rc=$rc $(( $(date +%s%3N) - t0 ))ms" >> $out/summary.txt
    [ $rc -ge 124 ] && exit $rc
  done
done
ALLRED_TEST_SHARE_GROUPS=2,4,8 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py -m gpu > $out/multi.log 2>&1; rc=$?; tail -3 $out/multi.log
cat $out/summary.txt
exit $rc
