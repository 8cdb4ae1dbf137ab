#!/bin/bash
# Kernel traces of multi-row decode steps (per-class duration and gaps, scripts/step_gaps.py).
set -u
OUT=${OUT:-gpurun_out/rtrace}
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "32" "8 --fp8" "64"; do
  tag=$(echo "$spec" | tr -d ' -')
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
    python3 scripts/trace_step.py --rows $spec --steps 20 > "$OUT/$tag.log" 2>&1 || { echo "FAILED $tag rc=$?"; exit 1; }
  f=$(ls "$OUT/$tag"/*/run_kernel_trace.csv 2>/dev/null || ls "$OUT/$tag"/run_kernel_trace.csv)
  python3 scripts/step_gaps.py $f 10 > "$OUT/gaps_$tag.txt" 2>&1
  cat "$OUT/gaps_$tag.txt"
  rm -f $f
done
