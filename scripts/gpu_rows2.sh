set -u
OUT=gpurun_out/${TAG:-rows2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_rows.py --rows 8,16,32 --profile-rows 32 > $OUT/rows32.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/rows32.log
timeout -k 10 300 python3 -u scripts/bench_rows.py --rows 8 --profile-rows 8 --fp8 > $OUT/rows8f.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/rows8f.log
