# round-5: which engine moves the chunked DMA path's 2D copies (kernel trace + memory-copy trace)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05l
mkdir -p $out
E2E_ARMS=dma_8 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d $out/tr -o run -- \
    python3 tools/e2e_probe.py 3 > $out/e2e.json 2> $out/e2e.err
rc=$?
cat $out/e2e.json
find $out -name "*stats.csv" | while read f; do echo "== $f"; cut -c1-160 "$f" | head -12; done
exit $rc
