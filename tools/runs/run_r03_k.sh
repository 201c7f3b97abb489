# round-3: where the schedule form's time goes — per-phase stamps (tools/steps_phases.py) and SQ counters
# of k_steps_pipe at config 2 (BO, LO); one --pmc pass of 8 SQ counters each
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03k
mkdir -p $out
for v in bo lo; do
  timeout -k 10 120 python tools/steps_phases.py $v >> $out/phases.jsonl 2>> $out/err || exit 1
done
cat $out/phases.jsonl
for v in "bo 5" "lo 320"; do
  tag=${v%% *}
  AB_EXEC=steps AB_EAGER=1 AB_SETS=32 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -f csv -d $out/sq_$tag -o run -- \
    python3 tools/ab_fused.py $v 50 > /dev/null 2>> $out/err || exit 1
  AB_EAGER=1 AB_SETS=32 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -f csv -d $out/sqf_$tag -o run -- \
    python3 tools/ab_fused.py $v 50 > /dev/null 2>> $out/err || exit 1
done
find $out -name "*counter_collection.csv"
