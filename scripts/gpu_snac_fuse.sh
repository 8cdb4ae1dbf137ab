# Fused depthwise -> pointwise SNAC stages: parity (SNAC, composed, batching, engine, service,
# long read), then window timings fused (default) vs MORPHEUS_MX_SNAC_FUSE=0, then the ordered
# single-window trace and the 7x32 per-grid summary.
set -u
OUT=gpurun_out/${TAG:-snac_fuse}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_snac.py tests/test_gpu_composed.py tests/test_gpu_batching.py tests/test_gpu_engine.py \
  tests/test_gpu_service.py tests/test_gpu_long_read.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python3 scripts/bench_snac.py > $OUT/snac_fused.log 2>&1 || exit $?
MORPHEUS_MX_SNAC_FUSE=0 timeout -k 10 300 python3 scripts/bench_snac.py > $OUT/snac_unfused.log 2>&1 || exit $?
echo fused; cat $OUT/snac_fused.log | grep N; echo unfused; cat $OUT/snac_unfused.log | grep N
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt1 -o kt -- python3 scripts/bench_snac.py --cases 7x1 --reps 3 > $OUT/kt1.log 2>&1 || exit $?
f=$(find $OUT/kt1 -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_order.py $f 28 > $OUT/order_7x1.txt
rm -f $f
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt32 -o kt -- python3 scripts/bench_snac.py --cases 7x32 --reps 3 > $OUT/kt32.log 2>&1 || exit $?
f=$(find $OUT/kt32 -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_by_grid.py $f --kernel mx:: > $OUT/by_grid_7x32.json
rm -f $f
cat $OUT/order_7x1.txt
