#!/bin/bash
# PMC records of the multi-row decode GEMMs, per projection kind: FETCH_SIZE, WRITE_SIZE and
# one 8-counter SQ pass, each its own rocprofv3 run (counter limits: MI355X_MICROARCH.md), over
# scripts/pmc_gemv.py (graph sweeps over all 28 layers' weights, no Infinity-Cache reuse) for
# 8 bf16 rows, 8 e4m3 rows and 32 bf16 rows; records built by scripts/pmc_rows_record.py.
set -u
OUT=${OUT:-gpurun_out/pmc_rows_kinds}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag args...
  local tag=$1; shift
  for pass in FETCH_SIZE WRITE_SIZE SQ; do
    local ctr=$pass
    [ $pass = SQ ] && ctr="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
    timeout -s KILL 200 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$tag.$pass -o $pass -- python3 scripts/pmc_gemv.py "$@" > $OUT/$tag.$pass.log 2>&1 || { echo "FAILED $tag $pass"; tail -5 $OUT/$tag.$pass.log; exit 1; }
    f=$(find $OUT/$tag.$pass -name '*counter_collection.csv' | head -1)
    python3 scripts/pmc_summary.py $f > $OUT/$tag.$pass.summary.jsonl
    rm -rf $OUT/$tag.$pass
  done
}
run rows8 --rows 8
run rows8fp8 --rows 8 --fp8
run rows32 --rows 32
python3 scripts/pmc_rows_record.py $OUT > $OUT/records.log && cat $OUT/records.log
