# round-3: the N > 1 bench path with 4 and 8 processes sharing the one GPU (peer transports, no RCCL)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh share 4 && bash tools/gpu.sh share 8
