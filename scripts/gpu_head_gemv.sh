# 2..8-row fp8 lm_head on the VALU GEMV (option head_gemv) vs the fp8 -> bf16 MFMA kernel:
# parity, then the 8-row fp8 decode step and the lm_head kernel times.
set -u
OUT=gpurun_out/${TAG:-head_gemv}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_fp8.py > $OUT/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -7
case $rc in 124|134|137|139) exit $rc;; esac
for o in 0 1; do
  timeout -k 10 120 python3 scripts/trace_step.py --rows 8 --fp8 --opt head_gemv=$o > $OUT/step_$o.log 2>&1 || exit $?
  grep ms/step $OUT/step_$o.log
done
timeout -k 10 120 python3 scripts/trace_step.py --rows 8 --fp8 > $OUT/step_0b.log 2>&1 || exit $?
grep ms/step $OUT/step_0b.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 scripts/trace_step.py --rows 8 --fp8 --opt head_gemv=1 > $OUT/kt.log 2>&1 || exit $?
find $OUT/kt -name '*kernel_trace.csv' -delete
f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1)
grep -E "gemv_kernel|gemm_rows_kernel<1, 1, 4" $f | cut -c1-200
