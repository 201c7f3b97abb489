# round-5: the chunked DMA end-to-end form (exactness at every chunk count), the multi-GPU CLI
# orchestration (groups sharing the GPU), then the N = 1 bench line (host_staged variants)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05b
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_multi.py -m gpu -q -rs -x --timeout 240 \
    --timeout-method thread > $out/tests.log 2>&1
rc=$?
tail -15 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?
tail -3 $out/bench.err
python -c "import json; d=json.load(open('$out/bench.json')); print(d['ms_per_step'], d['roofline']['frac'], json.dumps(d['host_staged']))"
exit $rc
