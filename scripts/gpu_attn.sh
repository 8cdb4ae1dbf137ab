set -u
OUT=gpurun_out/${TAG:-attn}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u scripts/pmc_attn.py --lens 64,128,256,512,600,1024,1200,2048 > $OUT/sweep.log 2>&1 || exit $?
timeout -k 10 200 python3 -u scripts/pmc_attn.py --lens 600,1200 --cpw 2 >> $OUT/sweep.log 2>&1 || exit $?
timeout -k 10 200 python3 -u scripts/pmc_attn.py --lens 600,1200 --cpw 1 >> $OUT/sweep.log 2>&1 || exit $?
grep '"rows"' $OUT/sweep.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d $OUT/sq -o sq -- python3 scripts/pmc_attn.py --lens 600 > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fs -o fs -- python3 scripts/pmc_attn.py --lens 600 > $OUT/fs.log 2>&1 || { tail -5 $OUT/fs.log; exit 1; }
for f in $(find $OUT -name '*counter_collection.csv'); do python3 scripts/pmc_summary.py $f --kernel attn_kernel > $f.summary.json; cat $f.summary.json; done
