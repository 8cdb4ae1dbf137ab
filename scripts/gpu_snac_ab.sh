# SNAC window timings + parity after a conv-GEMM change (ordered single-window trace kept).
set -u
OUT=gpurun_out/${TAG:-snac_ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_snac.py tests/test_gpu_composed.py tests/test_gpu_batching.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 scripts/bench_snac.py > $OUT/snac.log 2>&1 || exit $?
grep N $OUT/snac.log
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt1 -o kt -- python3 scripts/bench_snac.py --cases 7x1 --reps 3 > $OUT/kt1.log 2>&1 || exit $?
f=$(find $OUT/kt1 -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_order.py $f 37 > $OUT/order_7x1.txt
rm -f $f
cat $OUT/order_7x1.txt
