# round-5: the whole GPU suite with k_hier_ws in it, smoke, then the N > 1 bench rehearsed with
# 2 / 8 processes on the one GPU and --force-dist (peer_hier_ws among the candidates)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05h
mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rs --maxfail=5 --timeout 400 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?
tail -12 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 > $out/force_dist.json 2> $out/force_dist.err &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --share-gpu --steps 20 --warmup 5 > $out/share_n2.json 2> $out/share_n2.err &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29534 bench.py --gpus 8 --share-gpu --steps 20 --warmup 5 > $out/share_n8.json 2> $out/share_n8.err
rc=$?
for f in force_dist share_n2 share_n8; do
  python3 -c "
import json,sys
try:
    d=json.load(open('$out/$f.json')); x=d['xgmi']
    print('$f', d['value'], d['ms_per_step'], x['headline_transport'], x.get('dropped'), sorted(x['transport_quick_ms'].items(), key=lambda kv: kv[1])[:5])
except Exception as e: print('$f', 'no line', e)
"
done
exit $rc
