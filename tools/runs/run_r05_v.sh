# round-5: k_hier_ws with / without the writing waves' poll backoff vs k_hier_x2, 2 / 4 / 8 processes
# sharing the GPU (tools/hier_share_probe.py; a rehearsal: compares arms only)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05v
mkdir -p $out
for w in 2 4 8; do
  timeout -k 10 300 python tools/hier_share_probe.py $w 40 3 > $out/share_$w.json 2> $out/share_$w.err || exit 1
  python3 -c "import json; d=json.loads(open('$out/share_$w.json').read().strip().splitlines()[-1]); print($w, d['median'], d['peer_status'])"
done
