#!/bin/bash
# SQ counter passes over trace_step.py decode steps (ARGS), one rocprofv3 run per pass
# (counter limits: MI355X_MICROARCH.md), summarised per (kernel, grid) by pmc_summary.py.
set -u
OUT=${OUT:-gpurun_out/pmc_sq}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:---rows 8 --steps 4 --pos 600}
pass() {  # name counters...
  local name=$1; shift
  local ctrs=${*//,/ }
  timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/$name -o $name -- python3 scripts/trace_step.py $ARGS > $OUT/$name.log 2>&1 || { echo "FAILED $name"; tail -5 $OUT/$name.log; exit 1; }
  f=$(find $OUT/$name -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f > $OUT/$name.summary.jsonl
  rm -f $f
}
# PASSES="name:CTR1,CTR2 name2:CTR3" overrides the two default SQ passes
if [ -n "${PASSES:-}" ]; then
  for p in $PASSES; do pass ${p%%:*} ${p#*:}; done
else
  pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES
  pass mix SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA
fi
ls $OUT
