# round-3: k_broadcast after the tree — event timing of the probe's arms, then its rocprofv3 trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03g
mkdir -p $out
NO_PEER=1 timeout -k 10 120 python tools/bcast_probe.py 100 > $out/bp_ev.out 2> $out/bp_ev.err && cat $out/bp_ev.out &&
NO_PEER=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/bp3 -o run -- python3 tools/bcast_probe.py 100 > $out/bp3.out 2> $out/bp3.err
