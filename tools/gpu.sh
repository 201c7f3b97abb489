#!/bin/bash
# tools/gpu.sh <what> [args] — the GPU-box command lines of this repo, run as
#   /usr/local/graft/bin/gpurun --timeout <s> -- 'bash tools/gpu.sh <what>'
# Every GPU step has its own time limit and the steps are chained with &&:
# after a fault or a timeout nothing more runs on the GPU in that call.
#   test [pytest args]   pytest -m gpu (per-test thread timeouts), then smoke()
#   smoke                __graft_entry__.smoke()
#   bench [bench args]   bench.py (default: the driver's N = 1 line)
#   prof <tag>           rocprofv3 --kernel-trace --stats of bench.py --main-only,
#                        then FETCH_SIZE and WRITE_SIZE in separate --pmc passes
#   ab <v> "<tiles>" <tune a> <tune b> ...   tools/ab_fused.py arms interleaved (ALLRED_TUNE per arm)
#   skew ["<pads>"]      rank-row skew A/B of the config-2 fused pass
#   pmc_lo               PMC traffic of the fused LO pass, rocprofv3 stats of the schedule forms
#   share <n>            the N > 1 bench path rehearsed with n ranks on the one GPU
#                        (bench.py --share-gpu: peer transports, no RCCL; numbers mean nothing)
#   hier [steps rounds]  tools/hier_step.py: the hierarchical step's forms on one GPU (W = 1)
#   sweep                tools/sweep.py: every variant and form over the reference's size sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
what=$1
shift
case "$what" in
test)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --maxfail=20 --timeout 240 \
        --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
    rc=$?
    tail -25 gpurun_out/gpu_tests.log
    [ $rc -eq 0 ] && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
    ;;
smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
    ;;
bench)
    timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
    rc=$?
    tail -3 gpurun_out/bench.err
    cat gpurun_out/bench.json
    exit $rc
    ;;
prof)
    tag=${1:-prof}
    out=gpurun_out/$tag
    mkdir -p "$out"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$out/trace" -o run -- \
        python3 bench.py --main-only --steps 200 --warmup 20 > "$out/bench.json" 2> "$out/bench.err" &&
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$out/fetch" -o run -- \
        python3 bench.py --main-only --steps 100 --warmup 10 --eager > /dev/null 2> "$out/fetch.err" &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$out/write" -o run -- \
        python3 bench.py --main-only --steps 100 --warmup 10 --eager > /dev/null 2> "$out/write.err"
    rc=$?
    find "$out" -name "*.csv" | head -20
    exit $rc
    ;;
ab)
    # ab <bo|lo|mem> "<tiles list>" "<ALLRED_TUNE a>" "<ALLRED_TUNE b>" ... : tools/ab_fused.py
    # per size, the arms interleaved three times (32 rotating sets: cold HBM)
    variant=$1 sizes=$2
    shift 2
    for tiles in $sizes; do
        for rep in 1 2 3; do
            for arm in "$@"; do
                ALLRED_TUNE="$arm" AB_SETS=${AB_SETS:-32} timeout -k 10 120 python tools/ab_fused.py "$variant" "$tiles" \
                    >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit 1
            done
        done
    done
    python - <<'EOF'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/ab.jsonl")]
by = collections.defaultdict(list)
for r in rows:
    by[(r["variant"], r["bytes_per_rank"], r["env"].get("ALLRED_TUNE", ""))].append(r["us"])
for k, v in by.items():
    print(k, sorted(v))
EOF
    ;;
pmc_lo)
    # HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the fused Swing LO (k_lo_dag_reg)
    # and rocprofv3 stats of the schedule forms (k_steps_pipe) at config 2 -> gpurun_out/pmc_lo
    out=gpurun_out/pmc_lo
    mkdir -p "$out"
    export AB_EAGER=1 AB_SETS=32
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$out/lo_fetch" -o run -- \
        python3 tools/ab_fused.py lo 320 100 > /dev/null 2> "$out/e1" &&
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$out/lo_write" -o run -- \
        python3 tools/ab_fused.py lo 320 100 > /dev/null 2> "$out/e2" &&
    AB_EXEC=steps timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d "$out/steps_trace" -o run -- \
        python3 tools/ab_fused.py bo 5 200 > "$out/steps_bo.json" 2> "$out/e3" &&
    AB_EXEC=steps timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d "$out/steps_lo_trace" -o run -- \
        python3 tools/ab_fused.py lo 320 200 > "$out/steps_lo.json" 2> "$out/e4"
    ;;
skew)
    # skew "<pads in elements>": rank-row skew A/B of the config-2 fused pass (stride = n + pad)
    rm -f gpurun_out/pad.jsonl
    for rep in 1 2; do
        for pad in ${1:-0 64 128 256 512 1024 2048 4096}; do
            AB_PAD=$pad AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py bo 5 200 >> gpurun_out/pad.jsonl \
                2>> gpurun_out/pad.err || exit 1
        done
    done
    python - <<'EOF2'
import json, collections
by = collections.defaultdict(list)
for l in open("gpurun_out/pad.jsonl"):
    r = json.loads(l); by[int(r["env"]["AB_PAD"])].append(r["us"])
for k in sorted(by): print(k * 2, "B skew:", sorted(by[k]))
EOF2
    ;;
share)
    n=${1:-2}
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus "$n" --share-gpu --steps 20 --warmup 5 \
        > gpurun_out/share_n$n.json 2> gpurun_out/share_n$n.err
    rc=$?
    tail -5 gpurun_out/share_n$n.err
    cat gpurun_out/share_n$n.json
    exit $rc
    ;;
hier)
    timeout -k 10 300 python tools/hier_step.py ${1:-100} ${2:-3} > gpurun_out/hier_step.json 2> gpurun_out/hier_step.err
    rc=$?
    cat gpurun_out/hier_step.json
    exit $rc
    ;;
sweep)
    timeout -k 10 500 python -u tools/sweep.py > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err
    rc=$?
    tail -2 gpurun_out/sweep.err
    exit $rc
    ;;
*)
    echo "usage: $0 test|smoke|bench|prof|ab|skew|pmc_lo|share|hier|sweep" >&2
    exit 2
    ;;
esac
