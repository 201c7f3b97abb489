cd /root/repo && export TMPDIR=/tmp && OUT=gpurun_out/ab9 && mkdir -p $OUT
for r in 1 2; do for P in 64 128 192 256 320 448 1088 4160; do
  AB_PAD=$P AB_SETS=32 timeout -k 10 120 python tools/ab_fused.py bo 5 400 >> $OUT/ab.jsonl || exit 0
done; done
echo DONE > $OUT/done
