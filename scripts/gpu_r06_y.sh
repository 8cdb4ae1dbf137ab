#!/bin/bash
# round 6: one-row attention beyond 8 splits of 128 (L > 1024): 192-position splits on 6-wave
# (cpw 1) or 3-wave (cpw 2) blocks and 256 on 8-wave (cpw 1) against the default 4-wave cpw 2
set -o pipefail
OUT=gpurun_out/r06_y
mkdir -p $OUT
echo "== bf16" > $OUT/ab.log
timeout -k 10 300 python -u scripts/ab_decode.py --pos 1100,1400 --variants base,b1_61,b1_32,b1_81 >> $OUT/ab.log 2>&1 &&
echo "== e4m3" >> $OUT/ab.log &&
timeout -k 10 300 python -u scripts/ab_decode.py --fp8 --pos 1100,1400 --variants base,b1_61,b1_32,b1_81 >> $OUT/ab.log 2>&1
rc=$?
cat $OUT/ab.log
exit $rc
