# round-6: the RCCL-side N > 1 extras (link_probe, rccl_allreduce_comparator) run over torch's nccl backend
# with one rank (RCCL refuses two ranks on one device, so no --share-gpu rehearsal reaches them), and the
# 2-rank shared-GPU bench contract test
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${R06P_OUT:-r06p}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_multi.py -v -rs --timeout 300 --timeout-method thread \
    > $out/tests.log 2>&1
rc=$?
tail -5 $out/tests.log
exit $rc
