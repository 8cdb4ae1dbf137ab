#!/bin/bash
# round 6: PCM-only SNAC calls cut to the kept slice's receptive field (capi.hip snac_cut):
# SNAC + serving-path parity tests, then same-box timing against the previous library
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_r; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_snac.py tests/test_gpu_composed.py tests/test_gpu_batching.py tests/test_gpu_service.py -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
P=project_morpheus_amd/libmorpheus_mx_prev.so
for rnd in 1 2; do
  timeout -k 10 200 python -u scripts/bench_snac.py --cases 4x1,5x1,5x12,5x32,4x32 > $OUT/snac_new_$rnd.log 2>&1 || exit 1
  MORPHEUS_MX_LIB=$P timeout -k 10 200 python -u scripts/bench_snac.py --cases 4x1,5x1,5x12,5x32,4x32 > $OUT/snac_prev_$rnd.log 2>&1 || exit 1
done
timeout -k 10 300 python -u scripts/snac_share.py > $OUT/share_new.log 2>&1 || exit 1
MORPHEUS_MX_LIB=$P timeout -k 10 300 python -u scripts/snac_share.py > $OUT/share_prev.log 2>&1 || exit 1
for f in snac_new_2 snac_prev_2 share_new share_prev; do tail -n 6 $OUT/$f.log; done
