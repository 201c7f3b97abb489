# round-4: schedule-form per-phase device stamps at config 2 (k_steps_reg, BO 3 / LO 4 workgroups per CU):
# when each wave's first and second strips start / end, the step-0 (load) wait, the LDS chain, the stores
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04h
STEPS_GRID=768 timeout -k 10 120 python tools/steps_phases.py bo > gpurun_out/r04h/bo.json 2> gpurun_out/r04h/bo.err && \
STEPS_GRID=1024 timeout -k 10 120 python tools/steps_phases.py lo > gpurun_out/r04h/lo.json 2> gpurun_out/r04h/lo.err
rc=$?; cat gpurun_out/r04h/bo.json gpurun_out/r04h/lo.json; exit $rc
