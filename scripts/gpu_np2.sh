set -u
mkdir -p gpurun_out/np2
timeout -k 10 400 python -u -m pytest tests/test_gpu_snac.py tests/test_gpu_service.py -m gpu -q -p no:cacheprovider -x --timeout 170 --timeout-method thread > gpurun_out/np2/snac_tests.log 2>&1; tail -3 gpurun_out/np2/snac_tests.log
MORPHEUS_MX_LIB=project_morpheus_amd/libmorpheus_mx_np2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_llm.py -m gpu -q -p no:cacheprovider -x --timeout 170 --timeout-method thread -k "orpheus_width_32 or orpheus_width_64 or 20_rows or 40_rows" > gpurun_out/np2/tests.log 2>&1; tail -3 gpurun_out/np2/tests.log
timeout -k 10 300 python scripts/bench_rows.py --rows 8,32,64 --profile-rows 32 > gpurun_out/np2/np3.log 2>&1 || exit $?
MORPHEUS_MX_LIB=project_morpheus_amd/libmorpheus_mx_np2.so timeout -k 10 300 python scripts/bench_rows.py --rows 8,32,64 --profile-rows 32 > gpurun_out/np2/np2.log 2>&1 || exit $?
tail -n 5 gpurun_out/np2/np3.log gpurun_out/np2/np2.log
