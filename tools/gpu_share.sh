#!/bin/bash
# GPU session: the N>1 bench path with 2 and 4 processes sharing one GPU (--share-gpu:
# peer transports only, RCCL refuses two ranks on one device).  A rehearsal of the
# driver's multi-GPU run, not a measurement.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-share}
mkdir -p $OUT
for n in ${NS:-2 4}; do
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --share-gpu \
      ${EXTRAS:---no-extras} --steps 50 --warmup 5 > $OUT/bench_share$n.json 2> $OUT/bench_share$n.err
  rc=$?
  echo "N=$n EXIT $rc" >> $OUT/status
  [ $rc -eq 0 ] || exit 0
done
echo DONE > $OUT/done
