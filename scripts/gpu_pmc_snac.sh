# SNAC PMC record at 7 frames x 32 windows (the configs[2] shape): HBM bytes and SQ stall
# counters of the tiled conv-GEMM and the dwconv. Each counter set is its own rocprofv3 pass.
set -u
OUT=gpurun_out/pmc_snac
mkdir -p $OUT
export TMPDIR=/tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 scripts/bench_snac.py --cases 7x32 --reps 3 > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  f=$(find $OUT/$name -name '*counter_collection.csv' | head -1)
  python3 scripts/pmc_summary.py $f --kernel conv_gemm_tiled > $OUT/$name.tiled.json
  python3 scripts/pmc_summary.py $f --kernel dwconv > $OUT/$name.dwconv.json
  rm -f $f
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 scripts/bench_snac.py --cases 7x32 --reps 3 > $OUT/kt.log 2>&1
find $OUT/kt -name '*kernel_trace.csv' -delete
exit 0
