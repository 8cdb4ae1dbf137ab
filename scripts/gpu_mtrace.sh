set -u
OUT=gpurun_out/${TAG:-mtrace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/mega_trace.py ${ARGS:-} > $OUT/trace.log 2>&1 || exit $?
grep '^{' $OUT/trace.log
timeout -k 10 300 python -u scripts/mega_trace.py --fp8 ${ARGS:-} > $OUT/trace_fp8.log 2>&1 || exit $?
grep '^{' $OUT/trace_fp8.log
