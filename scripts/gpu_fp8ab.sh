set -u
export TMPDIR=/tmp
OUT=gpurun_out/fp8ab
mkdir -p $OUT
for R in 1 8 32; do
  timeout -k 10 300 python3 scripts/ab_decode.py --fp8 --rows $R --pos 600 --rounds 1 --variants base > $OUT/ab_fp8_r$R.log 2>&1; rc=$?
  echo "fp8 rows=$R: $(grep round $OUT/ab_fp8_r$R.log)"
  case $rc in 0) ;; *) tail -5 $OUT/ab_fp8_r$R.log; exit $rc;; esac
done
timeout -k 10 300 python3 scripts/ab_decode.py --rows 8 --pos 600 --rounds 1 --variants base > $OUT/ab_bf16_r8.log 2>&1; echo "bf16 rows=8: $(grep round $OUT/ab_bf16_r8.log)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o f -- python3 scripts/ab_decode.py --fp8 --rows 1 --pos 600 --rounds 1 --variants base > $OUT/prof.log 2>&1; rc=$?
find $OUT/prof -name '*kernel_trace.csv' -delete
exit $rc
