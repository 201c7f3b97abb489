#!/bin/bash
# GPU session: bench + kernel-trace profile + PMC traffic passes + tile-sum microbench.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r01}
mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o main --output-format csv -- python3 bench.py --main-only > $OUT/prof_main.log 2>&1 || exit 0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_tree_lds_lag -d $OUT/pmc_fetch -o fetch --output-format csv -- python3 bench.py --main-only --eager > $OUT/pmc_fetch.log 2>&1 || exit 0
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_tree_lds_lag -d $OUT/pmc_write -o write --output-format csv -- python3 bench.py --main-only --eager > $OUT/pmc_write.log 2>&1 || exit 0
timeout -k 10 300 python bench.py --force-dist --steps 50 --warmup 5 > $OUT/bench_forcedist.json 2> $OUT/bench_forcedist.err || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_forcedist -o fd --output-format csv -- python3 bench.py --force-dist --no-extras --steps 200 --warmup 20 > $OUT/prof_forcedist.log 2>&1 || exit 0
timeout -k 10 120 python tools/hier_local.py > $OUT/hier_local.json 2> $OUT/hier_local.err || exit 0
timeout -k 10 300 python tools/tilesum_bench.py > $OUT/tilesum.json 2> $OUT/tilesum.err || exit 0
echo DONE > $OUT/done
