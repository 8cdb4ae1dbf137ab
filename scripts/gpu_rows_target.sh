#!/bin/bash
# K-range target sweep of the multi-row GEMM (option rows_target; 0 = per-class default) and
# attention chunks per wave at 32 / 64 rows (att_cpw_batch; default auto = one split per row).
set -u
OUT=${OUT:-gpurun_out/rtarget}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  timeout -k 10 150 python3 scripts/trace_step.py "$@" --steps 20 >> "$OUT/sweep.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; tail -5 "$OUT/sweep.log"; exit 1; fi
}
for t in 0 256 384 512 768; do run --rows 32 --opt rows_target=$t; done
for t in 0 384 512; do run --rows 8 --fp8 --opt rows_target=$t; done
for t in 0 384 512 768; do run --rows 64 --opt rows_target=$t; done
for c in 1 2 4; do run --rows 32 --opt att_cpw_batch=$c; done
for c in 1 2; do run --rows 64 --opt att_cpw_batch=$c; done
grep "ms/step" "$OUT/sweep.log"
