#!/bin/bash
# round 6: option att_b1_short (one-row attention on 64 / 96-position splits): parity, then A/B
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_x; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread -k "short_splits or parity_orpheus or single_stream or split_classes or long_context_orpheus_width_default" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_decode.py --rows 1 --variants base,short1,short2 --pos 200,300,600,1100 --rounds 3 > $OUT/ab_r1.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_decode.py --rows 1 --fp8 --variants base,short1,short2 --pos 200,300,600,1100 --rounds 3 > $OUT/ab_r1f8.log 2>&1 || exit 1
tail -n 3 $OUT/ab_r1.log; tail -n 3 $OUT/ab_r1f8.log
