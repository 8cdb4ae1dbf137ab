#!/bin/bash
# Kernel traces of the decode step at several row counts (scripts/trace_step.py, L = 600):
# per kernel class the mean duration per step (scripts/step_gaps.py over the last 10 steps).
set -u
OUT=${OUT:-gpurun_out/step_traces}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in ${CFGS:-"r1:--rows 1" "r8:--rows 8" "r8fp8:--rows 8 --fp8" "r32:--rows 32"}; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- python3 scripts/trace_step.py $args ${EXTRA:-} > "$OUT/$tag.log" 2>&1 || { echo "FAILED $tag"; tail -5 "$OUT/$tag.log"; exit 1; }
  f=$(find "$OUT/$tag" -name '*kernel_trace.csv' | head -1)
  { grep ms/step "$OUT/$tag.log"; python3 scripts/step_gaps.py "$f" 10 commit_kernel; } > "$OUT/$tag.txt"
  cat "$OUT/$tag.txt" | head -14
  rm -rf "$OUT/$tag"
done
