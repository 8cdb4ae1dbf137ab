#!/bin/bash
# round 6: e4m3 one-row GEMV shapes; block order (rows_order) for prefill and 24 / 32 rows
set -o pipefail
O=gpurun_out/r06_l; mkdir -p $O
timeout -k 10 300 python -u scripts/ab_decode.py --rows 1 --fp8 --pos 600 --rounds 3 --reps 60 --variants base,ticket,wpb8,rpw_down2,wpb8_down2,rpw_gu2 > $O/ab_r1f8.log 2>&1 || exit 2
for o in 0 1 0 1; do
  timeout -k 10 200 python -u scripts/prefill_time.py --lens 64,256,512 --opt rows_order=$o >> $O/prefill.log 2>&1 || exit 3
done
timeout -k 10 300 python -u scripts/ab_decode.py --rows 32 --pos 600 --rounds 3 --reps 40 --variants base,order1 > $O/ab_r32.log 2>&1 || exit 4
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --pos 600 --rounds 3 --reps 40 --variants base,order1 > $O/ab_r8.log 2>&1 || exit 5
