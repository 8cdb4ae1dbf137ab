#!/bin/bash
# Prefill timings (bf16 / fp8 weights, 16..512 ids) and the round-3 PMC record of the 32-row
# projections (FETCH_SIZE and the SQ pass, scripts/pmc_gemv.py graph sweeps).
set -u
OUT=${OUT:-gpurun_out/prefill_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/prefill_time.py > $OUT/prefill_bf16.log 2>&1 || { tail -5 $OUT/prefill_bf16.log; exit 1; }
timeout -k 10 300 python3 scripts/prefill_time.py --fp8 > $OUT/prefill_fp8.log 2>&1 || { tail -5 $OUT/prefill_fp8.log; exit 1; }
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 scripts/pmc_gemv.py --rows 32 > $OUT/$name.log 2>&1 || { echo "FAILED $name"; tail -5 $OUT/$name.log; exit 1; }
  f=$(find $OUT/$name -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f --kernel gemm_rows > $OUT/$name.summary.json
  rm -f $f
}
pass r32_fetch FETCH_SIZE
pass r32_sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
grep -h '"n"' $OUT/prefill_*.log
