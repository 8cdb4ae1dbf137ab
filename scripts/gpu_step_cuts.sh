#!/bin/bash
# B = 1 dataflow step roles cut into per-layer launches (option step = 2, step_cuts mask:
# bit s starts a launch at stage s = qkv 0, attention 1, o-proj 2, gate/up 3, down 4) against
# the per-kernel hipGraph step (step = 0) and the one-launch step (step = 1).
set -u
OUT=${OUT:-gpurun_out/cuts}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  timeout -k 10 150 python3 scripts/trace_step.py "$@" --steps 50 >> "$OUT/sweep.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; tail -5 "$OUT/sweep.log"; exit 1; fi
}
run --opt step=0
run --opt step=1
for m in 1 9 25 27 29 31 3 5 17; do run --opt step=2 --opt step_cuts=$m; done
run --fp8 --opt step=0
for m in 1 9 25; do run --fp8 --opt step=2 --opt step_cuts=$m; done
grep "ms/step" "$OUT/sweep.log"
