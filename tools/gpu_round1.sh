#!/bin/bash
# GPU session: parity tests, bench, kernel-trace profile of the bench.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "PYTEST_EXIT $?" >> gpurun_out/pytest_gpu.log
rc=$(tail -1 gpurun_out/pytest_gpu.log | awk '{print $2}')
if [ "$rc" != "0" ]; then exit 0; fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo "DONE $?" >> gpurun_out/prof_bench.log
