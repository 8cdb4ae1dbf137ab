set -u
OUT=gpurun_out/r1e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o ab -- python3 scripts/ab_decode.py --rounds 1 --variants base --pos 2000 > $OUT/ab_prof.log 2>&1; rc=$?
for f in $(find $OUT/prof -name "*kernel_trace.csv"); do python3 scripts/trace_summary.py $f --bins 16 > $OUT/trace_summary.txt; rm -f $f; done
cat $OUT/trace_summary.txt
exit $rc
