set -u
OUT=gpurun_out/${TAG:-v7}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "batched or gen7 or gen4 or mega or persistent" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" $OUT/tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_rows.py --rows 8,16,32 --profile-rows 32 --options rows_kernel=7 > $OUT/rows7.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/rows7.log
timeout -k 10 300 python3 -u scripts/bench_rows.py --rows 8,16,32 --profile-rows 0 --options rows_kernel=4 > $OUT/rows4.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/rows4.log
for r in 8 16 32; do
  timeout -k 10 200 python -u scripts/mega_trace.py --ring $r > $OUT/trace_r$r.log 2>&1 || exit $?
  grep '^{' $OUT/trace_r$r.log
done
