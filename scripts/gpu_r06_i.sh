#!/bin/bash
# round 6: SNAC windows decoded as the frames the kept slice depends on (7 -> 5), noise keyed by
# position: serving-path parity against the full-window oracle, SNAC timings, configs[2] share
set -o pipefail
O=gpurun_out/r06_i; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_gpu_snac.py tests/test_gpu_composed.py tests/test_gpu_service.py tests/test_gpu_long_read.py tests/test_gpu_batching.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bench_snac.py --cases 1x1,4x1,7x1,5x1,7x12,5x12,7x32,5x32 > $O/bench_snac.log 2>&1 || exit 2
timeout -k 10 240 python -u scripts/snac_share.py > $O/snac_share.log 2>&1 || exit 3
