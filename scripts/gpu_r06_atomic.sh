#!/bin/bash
# round 6: engine give-up fix + rows_atomic A/B (bf16 8 / 32 rows, e4m3 8 rows; L 600)
set -o pipefail
O=gpurun_out/r06_atomic; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_engine_b1.py > $O/engine_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --pos 600 --rounds 3 --reps 50 --variants base,atomic,atomic_t384 > $O/ab_r8.log 2>&1 || exit 2
timeout -k 10 300 python -u scripts/ab_decode.py --rows 32 --pos 600 --rounds 3 --reps 50 --variants base,atomic,atomic_t384 > $O/ab_r32.log 2>&1 || exit 3
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --fp8 --pos 600 --rounds 3 --reps 50 --variants base,atomic,atomic_t384 > $O/ab_r8f8.log 2>&1 || exit 4
