#!/bin/bash
# round 6: K-range targets again at 24 / 32 rows under rows_nt1 = 2 (qkv / down on 32-row tiles)
set -o pipefail
O=gpurun_out/r06_h; mkdir -p $O
for rows in 32 24; do
  timeout -k 10 300 python -u scripts/ab_decode.py --rows $rows --pos 600 --rounds 3 --reps 40 --variants base,td256,td384,tq192,tq256,tgu384 > $O/ab_r$rows.log 2>&1 || exit 2
done
