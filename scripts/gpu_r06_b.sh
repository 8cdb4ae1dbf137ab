#!/bin/bash
# round 6: GPU suite with rows_atomic on by default; same-box A/B against the round-5 library
set -o pipefail
O=gpurun_out/r06_b; mkdir -p $O
R05=project_morpheus_amd/libmorpheus_mx_r05.so
for spec in "8:" "32:" "8:--fp8"; do
  rows=${spec%%:*}; f=${spec#*:}; tag=r${rows}${f:+f8}
  MORPHEUS_MX_LIB=$R05 timeout -k 10 200 python -u scripts/ab_decode.py --rows $rows $f --pos 600 --rounds 3 --reps 50 --variants base > $O/ab_${tag}_r05lib.log 2>&1 || exit 2
  timeout -k 10 200 python -u scripts/ab_decode.py --rows $rows $f --pos 600 --rounds 3 --reps 50 --variants seam,atomic > $O/ab_${tag}_new.log 2>&1 || exit 3
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
