# round-4: kernel traces of the in-process share-device rehearsal (allred_mem_2D, G = 4 groups on one GPU):
# do the failing runs' kernels start late (queue scheduling) or start together and wait (a protocol race)?
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04c
export ALLRED_TRANSPORT=peer ALLRED_SHARE_GPU=1 ALLRED_GPUS=4 ALLRED_NODES=4 GPU_MAX_HW_QUEUES=16 ALLRED_SHARE_SLOTS=256
mkdir -p $out
for i in 1 2 3 4 5 6; do
  t0=$(date +%s%3N)
  timeout -k 5 60 rocprofv3 --kernel-trace -f csv -d $out/run$i -o run -- tenstorrentallreduce_amd/bin/allred_mem_2D 1 1 2 13 40 32 \
    > $out/run$i.out 2> $out/run$i.err
  rc=$?
  echo "run$i rc=$rc $(( $(date +%s%3N) - t0 ))ms" >> $out/summary.txt
  [ $rc -ge 124 ] && exit $rc
done
exit 0
