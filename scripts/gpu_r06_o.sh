#!/bin/bash
# round 6: an attention change vs the previous library: multi-row parity tests, then same-box A/B (OUTD names the output)
set -u
export TMPDIR=/tmp
OUT=${OUTD:-gpurun_out/r06_o}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py tests/test_gpu_batching.py -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
OUT=$OUT/ab VARIANT_LIB=project_morpheus_amd/libmorpheus_mx_prev.so ROWS="1 8 32" bash scripts/gpu_ab_libs.sh || exit 1
OUT=$OUT/ab_f8 VARIANT_LIB=project_morpheus_amd/libmorpheus_mx_prev.so ROWS="8" F8=--fp8 bash scripts/gpu_ab_libs.sh || exit 1
