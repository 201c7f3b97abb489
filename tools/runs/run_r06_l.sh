# round-6: does the epoch-wrap test catch the advisor's case?  The same test against a library built with the
# round-5 rule (build/ab_oldwrap: a bucket larger than every entry is never checked) — [32] should fail there —
# then against the product library (both cases pass).  build/ab_oldwrap/liballred.so was built from this commit's
# tree with hier_area_prepare's check replaced by the round-5 rule (clear only when some staircase entry covers
# the new bucket: `if (covered && k - newest >= kHierWrapCalls)`), `make lib/liballred.so`, copied in place
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${R06L_OUT:-r06l}
mkdir -p $out
ALLRED_LIB_PATH=build/ab_oldwrap/liballred.so timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py \
    -k epoch_wrap -v --timeout 240 --timeout-method thread > $out/oldrule.log 2>&1
rc=$?
tail -6 $out/oldrule.log
# a failed assertion (rc 1) is the expected outcome; a timeout, a signal or a crash ends the call here
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -k epoch_wrap -v --timeout 240 --timeout-method thread \
    > $out/product.log 2>&1
rc=$?
tail -4 $out/product.log
exit $rc
