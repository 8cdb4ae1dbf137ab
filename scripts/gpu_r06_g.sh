#!/bin/bash
# round 6: batch-tile choice (rows_nt1) at 17-32 rows with the seam-free qkv / o-proj / down
set -o pipefail
O=gpurun_out/r06_g; mkdir -p $O
for rows in 32 24; do
  timeout -k 10 300 python -u scripts/ab_decode.py --rows $rows --pos 600 --rounds 3 --reps 40 --variants base,nt1_none,nt1_q,nt1_o,nt1_oq,nt1_d,nt1_od,nt1_qd > $O/ab_r$rows.log 2>&1 || exit 2
done
