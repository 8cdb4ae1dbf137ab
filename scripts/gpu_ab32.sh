set -u
OUT=${OUT:-gpurun_out/ab32}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 scripts/ab_decode.py --rows 32 --pos 600 --rounds 2 --variants base > $OUT/ab.log 2>&1; rc=$?
tail -3 $OUT/ab.log | head -2; grep round $OUT/ab.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o ab -- python3 scripts/ab_decode.py --rows 32 --pos 600 --rounds 1 --variants base > $OUT/ab_prof.log 2>&1; rc=$?
find $OUT/prof -name '*kernel_trace.csv' -delete
exit $rc
