# Per-launch durations of the SNAC kernels at 7 frames x 32 windows, by grid (pairs with the
# PMC passes of scripts/gpu_pmc_snac.sh, whose summaries are keyed by the same grid sizes).
set -u
OUT=gpurun_out/trace_snac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 scripts/bench_snac.py --cases 7x32 --reps 3 > $OUT/kt.log 2>&1 || exit $?
f=$(find $OUT/kt -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_by_grid.py $f > $OUT/by_grid.json
rm -f $f
cat $OUT/by_grid.json
