# round-4: schedule form with early loads only when the grid is full (steps_early auto): parity, then the size sweep
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04bb
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k "schedule_form" > gpurun_out/r04bb/parity.log 2>&1; rc=$?; tail -3 gpurun_out/r04bb/parity.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu.sh sweep
