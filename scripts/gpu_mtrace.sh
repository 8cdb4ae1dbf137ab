set -u
OUT=gpurun_out/${TAG:-mtrace}
mkdir -p $OUT
export TMPDIR=/tmp
for r in ${RINGS:-8 16 32}; do
  timeout -k 10 200 python -u scripts/mega_trace.py --ring $r ${ARGS:-} > $OUT/trace_r$r.log 2>&1 || exit $?
  grep '^{' $OUT/trace_r$r.log
done
timeout -k 10 300 python -u scripts/mega_ab.py --ring ${ABRING:-16} --rounds 2 > $OUT/ab.log 2>&1 || exit $?
grep '^{' $OUT/ab.log
