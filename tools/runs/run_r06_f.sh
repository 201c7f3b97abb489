# round-6: the bench with no flags (K = 200: graph replays for the headline, the secondary kernels behind a spin),
# and the N > 1 path with the RCCL comparator in the code (1-rank RCCL, 2 processes sharing the GPU)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06f
mkdir -p $out
timeout -k 10 500 python bench.py > $out/bench_default.json 2> $out/bench_default.err &&
timeout -k 10 500 python bench.py --force-dist --steps 20 --warmup 5 > $out/force_dist.json 2> $out/force_dist.err &&
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29571 bench.py --gpus 2 --share-gpu --steps 20 --warmup 5 > $out/share_n2.json 2> $out/share_n2.err
rc=$?
python3 -c "
import json; d=json.load(open('$out/bench_default.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['timing']['method'], d['hierarchical_step_w1']['k_hier_ws']['us_per_step'], d['hierarchical_step_w1']['k_hier_ws']['spin_covered_submission'], d['schedule_faithful']['us_per_step'])"
for f in force_dist share_n2; do
  [ -s $out/$f.json ] && python3 -c "
import json; d=json.loads(open('$out/$f.json').read().strip().splitlines()[-1])
x=d['xgmi']; print('$f', d['config']['transport'], d['ms_per_step'], x.get('dropped'), x['budget']['wall_s'], x['budget']['skipped_for_deadline'], x.get('rccl_allreduce_comparator'))"
done
exit $rc
