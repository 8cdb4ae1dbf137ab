#!/bin/bash
# round 6: options att_nw6 (6-wave multi-row attention blocks, the shortest split covering the
# context) and gemv_balance (one-row qkv / merging o-proj grids balanced over the CUs): their
# parity tests and the related sets, then same-process A/B
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_q; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread -k "six_wave or split_attention or straddling or 8_rows or gemv_balance or single_stream or split_classes" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_decode.py --rows 1 --variants base,balance --pos 300,600,1100 --rounds 3 > $OUT/ab_r1.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_decode.py --rows 1 --fp8 --variants base,balance --pos 300,600,1100 --rounds 3 > $OUT/ab_r1f8.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --variants base,nw6 --pos 300,600,700,1100 --rounds 3 > $OUT/ab_r8.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --fp8 --variants base,nw6 --pos 300,600,700,1100 --rounds 3 > $OUT/ab_r8f8.log 2>&1 || exit 1
tail -3 $OUT/ab_r1.log $OUT/ab_r1f8.log $OUT/ab_r8.log $OUT/ab_r8f8.log
