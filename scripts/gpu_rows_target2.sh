#!/bin/bash
# Fewer K ranges per multi-row GEMM (option rows_target below the per-class defaults) with the
# partials of up to 8 ranges loaded in one merge round.
set -u
OUT=${OUT:-gpurun_out/rtarget2}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  timeout -k 10 150 python3 scripts/trace_step.py "$@" --steps 20 >> "$OUT/sweep.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; tail -5 "$OUT/sweep.log"; exit 1; fi
}
for t in 0 32 64 96 128; do run --rows 32 --opt rows_target=$t; done
for t in 0 64 128; do run --rows 8 --fp8 --opt rows_target=$t; done
for t in 0 64 128; do run --rows 64 --opt rows_target=$t; done
for t in 0 64 128; do run --rows 16 --opt rows_target=$t; done
grep "ms/step" "$OUT/sweep.log"
