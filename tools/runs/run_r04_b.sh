# round-4: peer tests (k_hier_x / x2 with and without the chunked form); W = 1 A/B of the chunk
# bookkeeping; share-device probe over the workgroup slots the groups divide; multi tests (G = 2, 4)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04b
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_peer.py -m gpu > $out/peer.log 2>&1; rc=$?; tail -3 $out/peer.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  HIER_ARMS=hier_ll,hier_x,hier_x_ch,hier_x2,hier_x2_ch,hier_x2_tail,hier_x2_tail_ch timeout -k 10 120 \
    python tools/hier_step.py 200 3 >> $out/hier_chunk_ab.json 2>> $out/hier_step.err || exit 1
done
QUEUES="16 32" tools/multi_share_probe.sh $out/multi_share_probe.txt || exit 1
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py -m gpu > $out/multi.log 2>&1; rc=$?; tail -3 $out/multi.log
exit $rc
