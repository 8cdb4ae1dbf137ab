#!/bin/bash
# round 6: per-kernel step traces at 1 / 8 / 32 rows (bf16) and 1 / 8 rows (e4m3), L 600
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_traces; mkdir -p $OUT
run() {
  local tag=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- python3 scripts/trace_step.py "$@" > "$OUT/$tag.log" 2>&1 || { echo "FAILED $tag"; tail -5 "$OUT/$tag.log"; exit 1; }
  f=$(find "$OUT/$tag" -name '*kernel_trace.csv' | head -1)
  { grep ms/step "$OUT/$tag.log"; python3 scripts/step_gaps.py "$f" 10 commit_kernel; } > "$OUT/$tag.txt"
  rm -rf "$OUT/$tag"
}
run r1 --rows 1
run r1fp8 --rows 1 --fp8
run r8 --rows 8
run r8fp8 --rows 8 --fp8
run r32 --rows 32
