#!/bin/bash
# GPU session: full -m gpu suite, then bench + profiles (TAG names the output dir).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit 0
[ -n "$NOPROF" ] && exit 0
TAG=${TAG:-run} bash tools/gpu_prof.sh
