set -u
OUT=gpurun_out/${TAG:-pmcrows}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--rows ${ROWS:-32} --kinds ${KINDS:-gate_up,qkv} --options ${OPTS:-rows_kernel=4}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o sq -- python3 scripts/pmc_gemv.py $ARGS > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fs -o fs -- python3 scripts/pmc_gemv.py $ARGS > $OUT/fs.log 2>&1 || { tail -5 $OUT/fs.log; exit 1; }
for f in $(find $OUT -name '*counter_collection.csv'); do python3 scripts/pmc_summary.py $f --kernel gemm_rows > $f.summary.json; cat $f.summary.json; done
grep "us/launch" $OUT/sq.log
