#!/bin/bash
# Multi-row GEMM epilogue operands loaded before the split-K hand-off (default) vs after it
# (option rows_late_pre = 1), same box: parity tests, then step timings.
set -u
OUT=${OUT:-gpurun_out/preab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py tests/test_gpu_batching.py -m gpu -k "batched or rows or fp8 or batch" -v -p no:cacheprovider --timeout 170 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -3 "$OUT/tests.log"
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
for spec in "32" "8 --fp8" "64" "32" "8 --fp8"; do
  for s in 1 0; do
    timeout -k 10 150 python3 scripts/trace_step.py --rows $spec --steps 30 --opt rows_late_pre=$s >> "$OUT/steps.log" 2>&1 || { echo "FAILED $spec pre $s"; tail -5 "$OUT/steps.log"; exit 1; }
  done
done
grep "ms/step" "$OUT/steps.log"
