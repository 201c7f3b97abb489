# round-4: kernel trace + PMC traffic of the hierarchical forms with the round-4 placements (k_hier_x RE + late
# polls, k_hier_x2 TAIL 2 + late polls) next to the round-3 placements, W = 1
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04z
mkdir -p $out
export HIER_ARMS=hier_ll,hier_x,hier_x_re_lp,hier_x2_tail,hier_x2_tail2_lp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- python3 tools/hier_step.py 100 2 > $out/trace.json 2> $out/tr.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- python3 tools/hier_step.py 20 1 > /dev/null 2> $out/f.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- python3 tools/hier_step.py 20 1 > /dev/null 2> $out/w.err
