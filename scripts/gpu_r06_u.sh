#!/bin/bash
# round 6: SNAC block-tiled threshold re-checked on the receptive-field-cut shapes
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_u; mkdir -p $OUT
for rnd in 1 2; do
  for t in 8 4 16 33; do
    MORPHEUS_MX_SNAC_TILED_MIN_BATCH=$t timeout -k 10 200 python -u scripts/bench_snac.py --cases 5x1,5x4,5x8,5x12,5x16,5x32,4x8 > $OUT/t${t}_$rnd.log 2>&1 || exit 1
  done
done
for t in 8 4 16 33; do echo "== $t"; grep -h N5 $OUT/t${t}_2.log; grep -h N4 $OUT/t${t}_2.log; done
