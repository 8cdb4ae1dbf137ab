#!/bin/bash
# round 6: per-kind K-range targets with the seam-free qkv / o-proj / down
set -o pipefail
O=gpurun_out/r06_e; mkdir -p $O
V=base,tq192,tq256,tq384,td96,td256,td384,tgu384,to384
for spec in "8:" "32:" "8:--fp8" "16:"; do
  rows=${spec%%:*}; f=${spec#*:}; tag=r${rows}${f:+f8}
  timeout -k 10 300 python -u scripts/ab_decode.py --rows $rows $f --pos 600 --rounds 3 --reps 40 --variants $V > $O/ab_${tag}.log 2>&1 || exit 2
done
