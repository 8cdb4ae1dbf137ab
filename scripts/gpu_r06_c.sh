#!/bin/bash
# round 6: SNAC parity cases (mechanical coverage), SNAC MFMA / traffic record of the block-tiled
# conv-GEMM at 7 frames x 32 windows, one-row PMC traffic record of the current library.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06_c; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_snac.py > $O/snac_tests.log 2>&1 || exit 1
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o $name -- python3 scripts/bench_snac.py --cases 7x32 --reps 3 > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 2; }
  f=$(find $O/$name -name '*counter_collection.csv' | head -1)
  grep -E "^\"?[A-Za-z_]|conv_gemm_tiled" $f > $O/snac_$name.csv
  rm -f $f
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 scripts/bench_snac.py --cases 7x32 --reps 3 > $O/kt.log 2>&1 || exit 3
f=$(find $O/kt -name '*kernel_trace.csv' | head -1)
grep -E "^\"?[A-Za-z_]|conv_gemm_tiled" $f > $O/snac_kt.csv
rm -f $f
python3 scripts/snac_mfma_record.py $O/snac_kt.csv $O/snac_sq.csv $O/snac_fetch.csv $O/snac_write.csv > $O/r06_snac_mfma_record.json || exit 4
OUT=$O/pmc_b1 bash scripts/gpu_pmc_b1.sh > $O/pmc_b1.log 2>&1 || exit 5
