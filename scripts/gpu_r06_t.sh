#!/bin/bash
# round 6: prefill batch-tile cap (option rows_nt_max): 32-row tiles (2) vs 64-row (0 = 4) vs 16 (1)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_t; mkdir -p $OUT
for rnd in 1 2; do
  for o in 0 2 1; do
    timeout -k 10 240 python -u scripts/prefill_time.py --lens 24,48,64,128,256,512 --opt rows_nt_max=$o >> $OUT/prefill.log 2>&1 || exit 1
  done
done
timeout -k 10 240 python -u scripts/prefill_time.py --lens 24,48,64,128,256,512 --fp8 --opt rows_nt_max=0 >> $OUT/prefill.log 2>&1 || exit 1
timeout -k 10 240 python -u scripts/prefill_time.py --lens 24,48,64,128,256,512 --fp8 --opt rows_nt_max=2 >> $OUT/prefill.log 2>&1 || exit 1
grep -v amdgpu $OUT/prefill.log
