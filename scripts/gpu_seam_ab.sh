#!/bin/bash
# Split-K hand-off A/B for the multi-row GEMM (option rows_seam): parity (bitwise between the
# two, and against the oracle), then step timings at 32 / 64 / 8-fp8 / 16 rows for both.
set -u
OUT=${OUT:-gpurun_out/seamab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_llm.py -m gpu -k "tagged_seam or orpheus_width_32 or orpheus_width_64" -v -p no:cacheprovider --timeout 170 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -12 "$OUT/tests.log"
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
for spec in "32" "64" "8 --fp8" "16"; do
  for s in 0 1; do
    timeout -k 10 150 python3 scripts/trace_step.py --rows $spec --steps 20 --opt rows_seam=$s >> "$OUT/steps.log" 2>&1 || { echo "FAILED $spec seam $s"; tail -5 "$OUT/steps.log"; exit 1; }
  done
done
grep "ms/step" "$OUT/steps.log"
