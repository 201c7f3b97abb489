# round-4: schedule form staging only its units' block programs (tune steps_tab=1) vs every block's:
# parity of every schedule-form case, then A/B at config 2 (BO, 3 and 4 groups per CU)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04j
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k "schedule_form" > gpurun_out/r04j/parity.log 2>&1; rc=$?; tail -3 gpurun_out/r04j/parity.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.jsonl
AB_EXEC=steps bash tools/gpu.sh ab bo 5 steps_tab=0 steps_tab=1 "steps_tab=1,steps_groups=4" "steps_tab=0,steps_groups=4"
