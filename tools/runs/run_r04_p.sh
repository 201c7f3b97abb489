# round-4: final schedule form (per-unit program staging + early first-strip loads, LO program first):
# parity, rocprofv3 stats and PMC traffic of k_steps_reg BO / LO at config 2
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04p
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py -m gpu \
  -k "schedule_form" > $out/parity.log 2>&1; rc=$?; tail -3 $out/parity.log; [ $rc -eq 0 ] || exit $rc
AB_EXEC=steps timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/bo_trace -o run -- \
    python3 tools/ab_fused.py bo 5 200 > $out/steps_bo.json 2> $out/e1 && \
AB_EXEC=steps timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/lo_trace -o run -- \
    python3 tools/ab_fused.py lo 320 200 > $out/steps_lo.json 2> $out/e2 && \
AB_EXEC=steps timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch -o run -- \
    python3 tools/ab_fused.py bo 5 50 > /dev/null 2> $out/e3 && \
AB_EXEC=steps timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write -o run -- \
    python3 tools/ab_fused.py bo 5 50 > /dev/null 2> $out/e4 && \
AB_EXEC=steps timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/fetch_lo -o run -- \
    python3 tools/ab_fused.py lo 320 50 > /dev/null 2> $out/e5 && \
AB_EXEC=steps timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/write_lo -o run -- \
    python3 tools/ab_fused.py lo 320 50 > /dev/null 2> $out/e6
rc=$?; cat $out/steps_bo.json $out/steps_lo.json; exit $rc
