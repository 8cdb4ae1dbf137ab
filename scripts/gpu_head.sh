#!/bin/bash
# Multi-row lm_head study: launch time by rows x head option (bf16, e4m3), then FETCH_SIZE and
# an SQ pass over the 8-row head (scripts/pmc_gemv.py --kinds lm_head), each its own run.
set -u
OUT=${OUT:-gpurun_out/head}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/bench_head.py ${HEAD_ARGS:-} > $OUT/bf16.log 2>&1 || { tail -5 $OUT/bf16.log; exit 1; }
grep -v amdgpu.ids $OUT/bf16.log
timeout -k 10 240 python -u scripts/bench_head.py --fp8 ${HEAD_ARGS:-} > $OUT/fp8.log 2>&1 || { tail -5 $OUT/fp8.log; exit 1; }
grep -v amdgpu.ids $OUT/fp8.log
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
for pass in FETCH_SIZE SQ; do
  ctr=$pass
  [ $pass = SQ ] && ctr="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
  timeout -s KILL 200 rocprofv3 --pmc $ctr --output-format csv -d $OUT/h8.$pass -o $pass -- python3 scripts/pmc_gemv.py --rows 8 --kinds lm_head > $OUT/h8.$pass.log 2>&1 || { echo "FAILED $pass"; tail -5 $OUT/h8.$pass.log; exit 1; }
  f=$(find $OUT/h8.$pass -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f > $OUT/h8.$pass.summary.jsonl
  rm -rf $OUT/h8.$pass
  cat $OUT/h8.$pass.summary.jsonl
done
exit 0
