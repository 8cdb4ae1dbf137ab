#!/bin/bash
# round 6: option att_b1_nw6 (one-row 192-position splits past L 1,024) -- same-process A/B
# against att_b1_nw6 = 0, then every GPU parity test on the new default
set -o pipefail
OUT=gpurun_out/r06_z
mkdir -p $OUT
echo "== bf16" > $OUT/ab.log
timeout -k 10 300 python -u scripts/ab_decode.py --pos 900,1100,1400 --variants base,no_b1_nw6 >> $OUT/ab.log 2>&1 &&
echo "== e4m3" >> $OUT/ab.log &&
timeout -k 10 300 python -u scripts/ab_decode.py --fp8 --pos 900,1100,1400 --variants base,no_b1_nw6 >> $OUT/ab.log 2>&1 &&
cat $OUT/ab.log &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -n 5 $OUT/tests.log
exit $rc
