set -u
OUT=gpurun_out/${TAG:-snac}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_snac.py tests/test_gpu_engine.py -q -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 scripts/bench_snac.py > $OUT/snac.log 2>&1; rc=$?
cat $OUT/snac.log | grep N
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o snac -- python3 scripts/bench_snac.py > $OUT/snac_prof.log 2>&1; rc=$?
find $OUT/prof -name '*kernel_trace.csv' -delete
exit $rc
