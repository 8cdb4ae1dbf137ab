#!/bin/bash
# Round-3 PMC record of the one-launch B=1 decode step (bench roofline traffic): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes over scripts/trace_step.py, plus one SQ stall pass.
set -u
OUT=${OUT:-gpurun_out/pmc3}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:---steps 6 --pos 600}
pass() {  # name counters... -- (args from $ARGS)
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 scripts/trace_step.py $ARGS > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  f=$(find $OUT/$name -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f --kernel step_kernel > $OUT/$name.summary.jsonl
  rm -f $f
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES
python3 scripts/pmc_step_record.py $OUT "$ARGS" > $OUT/r03_pmc_step.json && cat $OUT/r03_pmc_step.json
