# round-4: BO schedule form with strips loaded two ahead into two register sets (tune steps_depth=2, 163 VGPRs):
# parity, then A/B at config 2 (BO 5 tiles), arms interleaved, twice
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04s
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k "schedule_form" > gpurun_out/r04s/parity.log 2>&1; rc=$?; tail -3 gpurun_out/r04s/parity.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.jsonl
AB_EXEC=steps bash tools/gpu.sh ab bo 5 steps_depth=1 steps_depth=2 > /dev/null && \
AB_EXEC=steps bash tools/gpu.sh ab bo 5 steps_depth=1 steps_depth=2 "steps_depth=2,steps_early=0"
