set -u
OUT=gpurun_out/${TAG:-rows}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K:-batched}" > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_rows.py --rows ${ROWS:-8,16,32} --profile-rows ${PROW:-32} ${OPTS:-} > $OUT/rows.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/rows.log
