#!/bin/bash
# GPU session: peer-transport tests + the N>1 bench path on one GPU (force-dist) + its kernel trace
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-peer}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_peer.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest_peer.log
[ $rc -eq 0 ] || exit 0
timeout -k 10 300 python bench.py --force-dist --no-extras --steps 100 --warmup 10 > $OUT/bench_forcedist.json 2> $OUT/bench_forcedist.err || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_fd -o fd --output-format csv -- python3 bench.py --force-dist --no-extras --steps 200 --warmup 20 > $OUT/prof_fd.log 2>&1 || exit 0
echo DONE > $OUT/done
