#!/bin/bash
# round 6: where a prefill's time goes (kernel trace of 256- and 48-id prefills)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_s; mkdir -p $OUT
for n in 256 48; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$n -o run -- python3 scripts/prefill_time.py --lens $n --reps 5 > $OUT/p$n.log 2>&1 || { echo "FAILED $n"; tail -5 $OUT/p$n.log; exit 1; }
  f=$(find $OUT/p$n -name '*kernel_stats.csv' | head -1)
  cp $f $OUT/p${n}_stats.csv
  find $OUT/p$n -name '*kernel_trace.csv' -delete
done
grep ms $OUT/p256.log $OUT/p48.log
