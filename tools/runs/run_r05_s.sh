# round-5: the N > 1 bench rehearsed on the final build (--force-dist, 4 processes sharing the GPU)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05s
mkdir -p $out
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 > $out/force_dist.json 2> $out/force_dist.err &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 4 --share-gpu --steps 20 --warmup 5 > $out/share_n4.json 2> $out/share_n4.err
rc=$?
for f in force_dist share_n4; do
  python3 -c "
import json
try:
    d=json.load(open('$out/$f.json')); x=d['xgmi']
    print('$f', d['value'], d['ms_per_step'], x['headline_transport'], x.get('dropped'), sorted(x['transport_quick_ms'].items(), key=lambda kv: kv[1])[:6])
except Exception as e: print('$f', 'no line', e)
"
done
exit $rc
