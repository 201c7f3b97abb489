# round-4: LO schedule form with every lane's partner / result rows read out of LDS once (tune steps_lo_rows):
# parity (schedule-form cases incl. capped grids), then A/B at config 2 (LO 320), arms interleaved, twice
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04r
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k "schedule_form" > gpurun_out/r04r/parity.log 2>&1; rc=$?; tail -3 gpurun_out/r04r/parity.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.jsonl
AB_EXEC=steps bash tools/gpu.sh ab lo 320 steps_lo_rows=0 steps_lo_rows=1 > /dev/null && \
AB_EXEC=steps bash tools/gpu.sh ab lo 320 steps_lo_rows=0 steps_lo_rows=1 "steps_lo_rows=1,steps_groups=3"
