# generation-8 multi-row GEMM: parity tests first, then rows sweep vs generation 4
set -u
mkdir -p gpurun_out/g8
timeout -k 10 600 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py tests/test_gpu_batching.py -m gpu -v -p no:cacheprovider -x --timeout 170 --timeout-method thread -k "batched or rows or fp8 or batch" > gpurun_out/g8/tests.log 2>&1; rc=$?
tail -5 gpurun_out/g8/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_rows.py --rows 8,16,32,64 --profile-rows 32 --options rows_gen=8 > gpurun_out/g8/g8.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_rows.py --rows 8,32 --profile-rows 8 --fp8 --options rows_gen=8 > gpurun_out/g8/g8_f8.log 2>&1 || exit $?
tail -n 6 gpurun_out/g8/g8.log gpurun_out/g8/g8_f8.log
timeout -k 10 300 python scripts/bench_rows.py --rows 8,16,32 --profile-rows 32 --options rows_gen=4 > gpurun_out/g8/g4.log 2>&1 || exit $?
tail -n 4 gpurun_out/g8/g4.log
