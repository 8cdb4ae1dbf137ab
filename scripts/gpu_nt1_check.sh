set -u
OUT=gpurun_out/nt1c; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab_decode.py --rows 32 --variants base,nt1_none --pos 300,600,1100 --rounds 2 > $OUT/r32.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_decode.py --rows 32 --fp8 --variants base,nt1_none --pos 600 --rounds 2 > $OUT/r32fp8.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py tests/test_gpu_sampling.py tests/test_gpu_long_read.py -m gpu -k "batched or straddl or rows or long_read or sampl" -q -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; for f in r32 r32fp8; do echo == $f; grep -hv round $OUT/$f.log | grep -v amdgpu; done; tail -3 $OUT/tests.log; exit $rc
