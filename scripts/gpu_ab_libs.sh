#!/bin/bash
# Same-box A/B of two library builds (product vs a build-time variant), interleaved processes:
#   VARIANT_LIB=project_morpheus_amd/libmorpheus_mx_<name>.so bash scripts/gpu_ab_libs.sh
set -u
OUT=${OUT:-gpurun_out/ab_libs}; mkdir -p $OUT
V=$VARIANT_LIB
ROWS=${ROWS:-"8 32"}
F8=${F8:-}   # "--fp8" for e4m3 weights
for rnd in 1 2; do
  for r in $ROWS; do
    timeout -k 10 200 python -u scripts/ab_decode.py --rows $r $F8 --variants base --pos 300,900 --rounds 1 > $OUT/prod_r${r}_$rnd.log 2>&1 || exit 1
    MORPHEUS_MX_LIB=$V timeout -k 10 200 python -u scripts/ab_decode.py --rows $r $F8 --variants base --pos 300,900 --rounds 1 > $OUT/var_r${r}_$rnd.log 2>&1 || exit 1
  done
done
if [ -n "${TESTS:-}" ]; then
  MORPHEUS_MX_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py -m gpu -k "$TESTS" -q -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log
fi
for r in $ROWS; do for rnd in 1 2; do echo "rows $r round $rnd prod: $(grep -h '^base' $OUT/prod_r${r}_$rnd.log)  var: $(grep -h '^base' $OUT/var_r${r}_$rnd.log)"; done; done
exit ${rc:-0}
