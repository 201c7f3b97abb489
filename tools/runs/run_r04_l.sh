# round-4: schedule form, per-unit program staging (steps_tab) x first strip's loads ahead (steps_early):
# parity, then A/B at config 2, BO (5 tiles) and LO (320), arms interleaved, twice
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04l
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k "schedule_form" > gpurun_out/r04l/parity.log 2>&1; rc=$?; tail -3 gpurun_out/r04l/parity.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.jsonl
for i in 1 2; do
  AB_EXEC=steps bash tools/gpu.sh ab bo 5 steps_tab=0 steps_tab=1 "steps_tab=1,steps_early=1" > /dev/null || exit 1
done
AB_EXEC=steps bash tools/gpu.sh ab lo 320 steps_tab=0 steps_early=1
