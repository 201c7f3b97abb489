# round-6: the N > 1 bench path rehearsed with its wall-clock budget (--deadline 420 s from the start of
# bench.py): a 1-rank RCCL communicator (--force-dist) and 2 / 4 / 8 processes sharing the GPU, each line
# recording xgmi.budget (phase seconds, total wall, skipped phases)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${R06D_OUT:-r06d}
mkdir -p $out
timeout -k 10 500 python bench.py --force-dist --steps 20 --warmup 5 > $out/force_dist.json 2> $out/force_dist.err &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29551 bench.py --gpus 2 --share-gpu --steps 20 --warmup 5 > $out/share_n2.json 2> $out/share_n2.err &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29552 bench.py --gpus 4 --share-gpu --steps 20 --warmup 5 > $out/share_n4.json 2> $out/share_n4.err &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29553 bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > $out/share_n8.json 2> $out/share_n8.err
rc=$?
for f in force_dist share_n2 share_n4 share_n8; do
  [ -s $out/$f.json ] && python3 -c "
import json; d=json.loads(open('$out/$f.json').read().strip().splitlines()[-1])
x=d['xgmi']; print('$f', d['config']['transport'], d['ms_per_step'], x.get('dropped'), json.dumps(x.get('budget'))[:900])"
done
exit $rc
