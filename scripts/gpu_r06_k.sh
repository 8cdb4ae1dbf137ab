#!/bin/bash
# round 6: e4m3 one-row GEMV shapes (verdict item 3)
set -o pipefail
O=gpurun_out/r06_k; mkdir -p $O
timeout -k 10 400 python -u scripts/ab_decode.py --rows 1 --fp8 --pos 300,600,1100 --rounds 3 --reps 60 --variants base,ticket,wpb8,rpw_down2,wpb8_down2,rpw_gu2 > $O/ab_r1f8.log 2>&1 || exit 2
