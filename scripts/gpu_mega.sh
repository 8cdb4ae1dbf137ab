set -u
OUT=gpurun_out/${TAG:-mega}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K:-mega or persistent or orpheus_width_2}" > $OUT/tests.log 2>&1; rc=$?
tail -25 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/mega_ab.py > $OUT/ab_bf16.log 2>&1 || exit $?
grep '^{' $OUT/ab_bf16.log
timeout -k 10 300 python -u scripts/mega_ab.py --fp8 > $OUT/ab_fp8.log 2>&1 || exit $?
grep '^{' $OUT/ab_fp8.log
