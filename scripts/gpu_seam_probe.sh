#!/bin/bash
# Price of the multi-row GEMM's split-K seam: per-class us/launch (graph sweeps over all 28
# layers, scripts/pmc_gemv.py) with and without the ticket + last-arriver merge (option
# rows_probe = 1: ranges publish their partials and exit; results invalid, timing only).
set -u
OUT=${OUT:-gpurun_out/seam}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rows in 32 8 64; do
  for p in 0 1; do
    echo "== rows $rows rows_probe $p" >> "$OUT/seam.log"
    timeout -k 10 150 python3 scripts/pmc_gemv.py --rows $rows --options rows_probe=$p >> "$OUT/seam.log" 2>&1 || { echo "FAILED rows $rows probe $p"; exit 1; }
  done
done
grep -v amdgpu.ids "$OUT/seam.log"
