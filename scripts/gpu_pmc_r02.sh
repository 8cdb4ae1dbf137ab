# Round-2 PMC record: HBM bytes of the one-row GEMVs (bench roofline traffic) and of the
# 32-row generation-4 GEMM on fragment-major weights, plus the 32-row SQ stall counters.
# Each counter set is its own rocprofv3 pass under a hard time limit.
set -u
OUT=gpurun_out/pmc2
mkdir -p $OUT
export TMPDIR=/tmp
pass() {  # name counters... -- args
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  timeout -s KILL 150 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d $OUT/$name -o $name -- python3 scripts/pmc_gemv.py "$@" > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
}
pass b1_fetch FETCH_SIZE -- --rows 1
pass b1_write WRITE_SIZE -- --rows 1
pass r32_fetch FETCH_SIZE -- --rows 32
pass r32_sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -- --rows 32
for n in b1_fetch b1_write; do
  f=$(find $OUT/$n -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f --kernel gemv1 > $OUT/$n.summary.json
  rm -f $f
done
for n in r32_fetch r32_sq; do
  f=$(find $OUT/$n -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f --kernel gemm_rows > $OUT/$n.summary.json
  rm -f $f
done
grep -h "us/launch" $OUT/*.log | head -20
