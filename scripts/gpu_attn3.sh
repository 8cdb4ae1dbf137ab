set -u
OUT=gpurun_out/${TAG:-attn3}
mkdir -p $OUT
export TMPDIR=/tmp
A="timeout -k 10 200 python3 -u scripts/pmc_attn.py"
{ $A --lens 1100,1200,1500 --cpw 6 && $A --lens 1100,1200,1500,2048 --cpw 4 && $A --lens 2048 --cpw 8 \
  && $A --lens 1200 --cpw 1 && $A --rows 16 --lens 1200,2048 --cpw 3 && $A --rows 16 --lens 2048 --cpw 6 ; } > $OUT/sweep.log 2>&1 || exit $?
grep '"rows"' $OUT/sweep.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_llm.py -k "chunk_counts or batched" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep -o '"configs_2_batched.*' $OUT/bench.log | cut -c1-1200
