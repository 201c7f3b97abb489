# round-4: schedule-form grid A/B at config 2 (pipe_grid: workgroups of k_steps_reg; 0 = 3 per CU = 768;
# 640 = exactly 2 strips per wave; 512 = 2 per CU; 1024 = 4 per CU at the 3-per-CU register budget)
set -o pipefail
export TMPDIR=/tmp
AB_EXEC=steps bash tools/gpu.sh ab bo 5 pipe_grid=0 pipe_grid=640 pipe_grid=512 pipe_grid=1024 && \
AB_EXEC=steps bash tools/gpu.sh ab lo 320 pipe_grid=0 pipe_grid=640 pipe_grid=1024 steps_groups=4
