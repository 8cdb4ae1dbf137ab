#!/bin/bash
# round 6: configs[2] SNAC window coalescing (MORPHEUS_MX_SNAC_MIN_BATCH / _MAX_HOLD) and the
# tiled threshold (MORPHEUS_MX_SNAC_TILED_MIN_BATCH) re-swept after the receptive-field cut,
# scripts/snac_share.py (32 streams x 1200 tokens, SNAC on / off), same box
set -u
export TMPDIR=/tmp
OUT=${OUTD:-gpurun_out/r06_w}; mkdir -p $OUT
for cfg in 16:3:8 16:3:12 12:2:8 24:4:8 16:3:8 16:3:12 12:2:8 24:4:8; do
  IFS=: read mb mh tt <<< "$cfg"
  MORPHEUS_MX_SNAC_MIN_BATCH=$mb MORPHEUS_MX_SNAC_MAX_HOLD=$mh MORPHEUS_MX_SNAC_TILED_MIN_BATCH=$tt timeout -k 10 300 python -u scripts/snac_share.py > $OUT/share_${mb}_${mh}_${tt}.log 2>&1 || exit 1
  echo "== min_batch $mb max_hold $mh tiled_min $tt"; grep -v amdgpu $OUT/share_${mb}_${mh}_${tt}.log
done
