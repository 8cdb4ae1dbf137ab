#!/bin/bash
# Attention K/V loads: default policy vs non-temporal (option att_nt), same box.
set -u
OUT=${OUT:-gpurun_out/attnt}
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "32" "1" "8 --fp8" "32" "1" "64"; do
  for s in 0 1; do
    timeout -k 10 150 python3 scripts/trace_step.py --rows $spec --steps 30 --opt att_nt=$s >> "$OUT/steps.log" 2>&1 || { echo "FAILED $spec nt $s"; tail -5 "$OUT/steps.log"; exit 1; }
  done
done
grep "ms/step" "$OUT/steps.log"
