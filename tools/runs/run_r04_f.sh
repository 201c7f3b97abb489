# round-4: schedule form with the first strip's loads ahead of the program staging (tune steps_early):
# parity (every schedule-form case), then A/B at config 2 (BO 5 tiles = 640 kB, LO 320), arms interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k "schedule_form" > gpurun_out/r04f/parity.log 2>&1; rc=$?; tail -3 gpurun_out/r04f/parity.log; [ $rc -eq 0 ] || exit $rc
AB_EXEC=steps bash tools/gpu.sh ab bo 5 steps_early=0 steps_early=1 && AB_EXEC=steps bash tools/gpu.sh ab lo 320 steps_early=0 steps_early=1
