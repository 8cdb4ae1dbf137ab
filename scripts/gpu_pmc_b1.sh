#!/bin/bash
# PMC traffic record of the one-row decode GEMVs (the bench roofline's `traffic`):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over scripts/pmc_gemv.py --rows 1.
set -u
OUT=${OUT:-gpurun_out/pmc_b1}
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o $c -- python3 scripts/pmc_gemv.py --rows 1 --kinds qkv,o_proj,o_proj_merge,gate_up,down,lm_head > $OUT/$c.log 2>&1 || { echo "FAILED $c"; tail -5 $OUT/$c.log; exit 1; }
  f=$(find $OUT/$c -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f > $OUT/$c.summary.json
  rm -f $f
done
python3 scripts/pmc_gemv_record.py $OUT/FETCH_SIZE.summary.json $OUT/WRITE_SIZE.summary.json $OUT/pmc_gemv.json "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes, scripts/gpu_pmc_b1.sh) over scripts/pmc_gemv.py --rows 1: one graph sweep of all 28 layers per GEMV (no Infinity-Cache reuse), bf16; hbm_read_bytes = FETCH_SIZE x 1024 x 2 (gfx950 correction, MI355X_MICROARCH.md HBM), hbm_write_bytes = WRITE_SIZE x 1024; medians"
