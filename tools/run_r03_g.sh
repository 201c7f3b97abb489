# round-3: k_broadcast after the tree — which of source / destination / launch mode / peer windows costs
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03g
mkdir -p $out
NO_PEER=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/bp_nopeer -o run -- python3 tools/bcast_probe.py 100 > $out/bp2.out 2> $out/bp2.err
