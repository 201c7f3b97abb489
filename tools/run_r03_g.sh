# round-3: k_broadcast after the tree (eager) — which of source / destination / launch mode costs
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03g
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/bp -o run -- python3 tools/bcast_probe.py 100 > $out/bp.out 2> $out/bp.err
