# round-5: the N > 1 bench path rehearsed — a 1-rank RCCL communicator (--force-dist: RCCL and rccl_x
# verified and timed first, then the peer candidates and fenced twins) and 2 / 4 processes sharing the GPU
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05e
mkdir -p $out
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 > $out/force_dist.json 2> $out/force_dist.err &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --share-gpu --steps 20 --warmup 5 > $out/share_n2.json 2> $out/share_n2.err &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29534 bench.py --gpus 4 --share-gpu --steps 20 --warmup 5 > $out/share_n4.json 2> $out/share_n4.err
rc=$?
for f in force_dist share_n2 share_n4; do
  python3 -c "
import json,sys
try:
    d=json.load(open('$out/$f.json')); x=d['xgmi']
    print('$f', d['value'], d['ms_per_step'], x['headline_transport'], x.get('dropped'), sorted(x['transport_quick_ms'].items(), key=lambda kv: kv[1])[:4])
except Exception as e: print('$f', 'no line', e)
"
done
exit $rc
