# round-4: schedule form with the step-0 pairs as kernel arguments (tune steps_pairs_arg): parity, then A/B
# at config 2 (BO 5 tiles, LO 320), arms interleaved, twice
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k "schedule_form" > gpurun_out/r04aa/parity.log 2>&1; rc=$?; tail -3 gpurun_out/r04aa/parity.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.jsonl
AB_EXEC=steps bash tools/gpu.sh ab bo 5 steps_pairs_arg=0 steps_pairs_arg=1 > /dev/null && \
AB_EXEC=steps bash tools/gpu.sh ab lo 320 steps_pairs_arg=0 steps_pairs_arg=1 > /dev/null && \
AB_EXEC=steps bash tools/gpu.sh ab bo 5 steps_pairs_arg=0 steps_pairs_arg=1 > /dev/null && \
AB_EXEC=steps bash tools/gpu.sh ab lo 320 steps_pairs_arg=0 steps_pairs_arg=1
