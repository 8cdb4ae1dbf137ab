set -u
OUT=gpurun_out/${TAG:-r1b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_llm.py tests/test_gpu_engine.py -q -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 scripts/bench_attention.py > $OUT/att.log 2>&1; rc=$?
tail -8 $OUT/att.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python3 scripts/ab_decode.py ${AB_ARGS:-} > $OUT/ab.log 2>&1; rc=$?
tail -40 $OUT/ab.log
exit $rc
