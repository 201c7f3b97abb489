# round-5: the N = 1 bench line with the W = 1 hierarchical step (k_hier_ws / k_hier_x2) in it
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05r
mkdir -p $out
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?
tail -3 $out/bench.err
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['hierarchical_step_w1'])"
exit $rc
