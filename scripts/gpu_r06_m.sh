#!/bin/bash
# round 6: attention staging with every qkv range's loads issued at once + LDS-typed q reads;
# multi-row parity, then A/B (qkv seam vs parts; block order), prefill order, e4m3 one-row shapes
set -o pipefail
O=gpurun_out/r06_m; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_llm.py tests/test_gpu_fp8.py -k "batched or straddl" > $O/rows_tests.log 2>&1 || exit 1
for spec in "8:" "32:" "8:--fp8"; do
  rows=${spec%%:*}; f=${spec#*:}; tag=r${rows}${f:+f8}
  timeout -k 10 200 python -u scripts/ab_decode.py --rows $rows $f --pos 600 --rounds 3 --reps 40 --variants qkvseam,base,order1 > $O/ab_${tag}.log 2>&1 || exit 2
done
for o in 0 1 0 1; do
  timeout -k 10 200 python -u scripts/prefill_time.py --lens 64,256,512 --opt rows_order=$o >> $O/prefill.log 2>&1 || exit 3
done
timeout -k 10 300 python -u scripts/ab_decode.py --rows 1 --fp8 --pos 600 --rounds 3 --reps 60 --variants base,ticket,wpb8,rpw_down2,wpb8_down2,rpw_gu2 > $O/ab_r1f8.log 2>&1 || exit 4
