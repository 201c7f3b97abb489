set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03g
mkdir -p $out
for r in 1 2; do NO_PEER=1 timeout -k 10 120 python tools/bcast_probe.py 200 >> $out/bp_ev2.out 2>> $out/bp_ev2.err || exit 1; done; cat $out/bp_ev2.out
