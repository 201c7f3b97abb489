# round-3: the schedule form's new kernel (k_steps_reg) — rocprofv3 kernel stats and PMC HBM traffic (separate
# --pmc passes) for BO (config 2) and LO (640 kB), then the reference's size sweep (tools/sweep.py)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03r
mkdir -p $out
export AB_SETS=32
for v in "bo 5" "lo 320"; do
  tag=${v%% *}
  AB_EXEC=steps timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $out/${tag}_trace -o run -- \
      python3 tools/ab_fused.py $v 200 > $out/${tag}_trace.json 2>> $out/err || exit 1
  AB_EXEC=steps AB_EAGER=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $out/${tag}_fetch -o run -- \
      python3 tools/ab_fused.py $v 100 > /dev/null 2>> $out/err || exit 1
  AB_EXEC=steps AB_EAGER=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $out/${tag}_write -o run -- \
      python3 tools/ab_fused.py $v 100 > /dev/null 2>> $out/err || exit 1
done
find $out -name "*.csv" | sort
timeout -k 10 500 python -u tools/sweep.py > $out/sweep.jsonl 2> $out/sweep.err; rc=$?; tail -2 $out/sweep.err; exit $rc
