#!/bin/bash
# lm_head change check: kernel times, block timeline of the head, multi-row parity tests.
set -u
OUT=${OUT:-gpurun_out/head_check}; mkdir -p $OUT
timeout -k 10 200 python -u scripts/bench_head.py --variants base > $OUT/bf16.log 2>&1 && \
timeout -k 10 200 python -u scripts/bench_head.py --fp8 --variants base > $OUT/fp8.log 2>&1 && \
timeout -k 10 200 python -u scripts/rows_block_trace.py --kinds lm_head > $OUT/trace.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py tests/test_gpu_sampling.py -m gpu -k "batched or straddl or rows or head or sampl" -x -q -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -h variant $OUT/bf16.log $OUT/fp8.log; grep -h rows $OUT/trace.log | cut -c1-400; tail -2 $OUT/tests.log; exit $rc
