#!/bin/bash
# Multi-row step A/B at 8 bf16 / 8 e4m3 / 32 bf16 rows (scripts/ab_decode.py), VARIANTS env.
set -u
OUT=${OUT:-gpurun_out/ab_rows}; mkdir -p $OUT
V=${VARIANTS:-base}
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --variants $V --pos 600 --rounds 2 > $OUT/r8.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --fp8 --variants $V --pos 600 --rounds 2 > $OUT/r8fp8.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_decode.py --rows 32 --variants $V --pos 600 --rounds 2 > $OUT/r32.log 2>&1
rc=$?; for f in r8 r8fp8 r32; do echo "== $f"; grep -v amdgpu $OUT/$f.log | grep -v round; done; exit $rc
