#!/bin/bash
# Multi-row attention at long contexts: the one-split auto choice (att_cpw_batch 0: up to 6-8
# chunks per wave in sequence) vs three chunks per wave over two or more splits (3).
set -u
OUT=${OUT:-gpurun_out/attlong}
mkdir -p "$OUT"
export TMPDIR=/tmp
for pos in 1200 900 1200; do
  for c in 0 3 2; do
    timeout -k 10 200 python3 scripts/trace_step.py --rows 32 --pos $pos --steps 20 --opt att_cpw_batch=$c >> "$OUT/steps.log" 2>&1 || { echo "FAILED pos $pos cpw $c"; tail -5 "$OUT/steps.log"; exit 1; }
  done
done
for c in 0 3; do
  timeout -k 10 200 python3 scripts/trace_step.py --rows 8 --fp8 --pos 1200 --steps 20 --opt att_cpw_batch=$c >> "$OUT/steps.log" 2>&1 || exit 1
done
grep "ms/step" "$OUT/steps.log"
