set -u
OUT=gpurun_out/${TAG:-mega2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "mega or persistent" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/mega_trace.py --ring 16 > $OUT/trace_r16.log 2>&1 || exit $?
grep '^{' $OUT/trace_r16.log
timeout -k 10 300 python -u scripts/mega_ab.py --ring 16 --rounds 2 > $OUT/ab.log 2>&1 || exit $?
grep '^{' $OUT/ab.log
timeout -k 10 300 python -u scripts/mega_ab.py --ring 16 --rounds 2 --fp8 > $OUT/ab8.log 2>&1 || exit $?
grep '^{' $OUT/ab8.log
