#!/bin/bash
# round 6: qkv_parts attention without the register patch (late first-chunk load): parity,
# A/B against the seam qkv, step traces
set -o pipefail
O=gpurun_out/r06_f; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_llm.py tests/test_gpu_fp8.py -k "batched or straddl" > $O/rows_tests.log 2>&1 || exit 1
for spec in "8:" "32:" "8:--fp8"; do
  rows=${spec%%:*}; f=${spec#*:}; tag=r${rows}${f:+f8}
  timeout -k 10 200 python -u scripts/ab_decode.py --rows $rows $f --pos 600 --rounds 3 --reps 50 --variants qkvseam,base > $O/ab_${tag}.log 2>&1 || exit 2
done
