#!/bin/bash
# lm_head K split at 32 / 8-fp8 rows (option rows_head_target: 0 = one range, 2048 -> 2 ranges,
# 4096 -> 4 ranges), same box, plus parity of the split head.
set -u
OUT=${OUT:-gpurun_out/headsplit}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_llm.py -m gpu -k "lm_head_k_split" -v -p no:cacheprovider --timeout 170 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -4 "$OUT/tests.log"
case $rc in 0) ;; *) echo "tests rc=$rc: stopping"; exit $rc;; esac
for spec in "32" "8 --fp8" "32" "8 --fp8"; do
  for t in 0 2048 4096; do
    timeout -k 10 150 python3 scripts/trace_step.py --rows $spec --steps 30 --opt rows_head_target=$t >> "$OUT/steps.log" 2>&1 || { echo "FAILED $spec $t"; tail -5 "$OUT/steps.log"; exit 1; }
  done
done
grep "ms/step" "$OUT/steps.log"
