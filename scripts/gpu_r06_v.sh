#!/bin/bash
# round 6: SNAC + serving-path parity after the tiled-threshold change; SNAC timing
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_v; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_snac.py tests/test_gpu_composed.py tests/test_gpu_batching.py tests/test_gpu_service.py -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_snac.py --cases 5x1,4x1,5x8,5x12,5x32 > $OUT/snac.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/snac_share.py > $OUT/share.log 2>&1 || exit 1
grep -v amdgpu $OUT/snac.log $OUT/share.log
