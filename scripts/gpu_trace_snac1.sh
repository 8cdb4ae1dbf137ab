# Ordered per-launch durations of one single-window (7 frames x 1) SNAC decode (graph replay),
# plus the 7x32 per-grid summary; baseline for the dwconv -> 1x1 fusion.
set -u
OUT=gpurun_out/${TAG:-trace_snac1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/bench_snac.py > $OUT/snac.log 2>&1 || exit $?
cat $OUT/snac.log
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt1 -o kt -- python3 scripts/bench_snac.py --cases 7x1 --reps 3 > $OUT/kt1.log 2>&1 || exit $?
f=$(find $OUT/kt1 -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_order.py $f 40 > $OUT/order_7x1.txt
rm -f $f
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt32 -o kt -- python3 scripts/bench_snac.py --cases 7x32 --reps 3 > $OUT/kt32.log 2>&1 || exit $?
f=$(find $OUT/kt32 -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_by_grid.py $f > $OUT/by_grid_7x32.json
rm -f $f
cat $OUT/order_7x1.txt
