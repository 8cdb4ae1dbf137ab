#!/bin/bash
# PMC record of the multi-row decode step (default 32 rows at L = 600): FETCH_SIZE, WRITE_SIZE
# and one SQ pass, each its own rocprofv3 run (counter limits: MI355X_MICROARCH.md), summarised
# per (kernel, grid) by scripts/pmc_summary.py.
set -u
OUT=${OUT:-gpurun_out/pmc_rows}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:---rows 32 --steps 4 --pos 600}
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 scripts/trace_step.py $ARGS > $OUT/$name.log 2>&1 || { echo "FAILED $name"; tail -5 $OUT/$name.log; exit 1; }
  f=$(find $OUT/$name -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f > $OUT/$name.summary.jsonl
  rm -f $f
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES
ls -la $OUT
