#!/bin/bash
# round 6: multi-row attention shape with the qkv_parts staging / atomic o-proj (8, 16 rows)
set -o pipefail
O=gpurun_out/r06_j; mkdir -p $O
for spec in "8:" "8:--fp8" "16:"; do
  rows=${spec%%:*}; f=${spec#*:}; tag=r${rows}${f:+f8}
  timeout -k 10 300 python -u scripts/ab_decode.py --rows $rows $f --pos 300,600,1100 --rounds 3 --reps 40 --variants base,cpwb2,cpwb4,cpwb6,nwb4,tmerge > $O/ab_${tag}.log 2>&1 || exit 2
done
