# SNAC one-wave conv-GEMM wave target / 16-wave tiles (MORPHEUS_MX_SNAC_WAVES, _WK_MAX) A/B.
set -u
OUT=gpurun_out/${TAG:-snac_wk}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "2048 8" "4096 16" "4096 8" "8192 16"; do
  set -- $cfg
  MORPHEUS_MX_SNAC_WAVES=$1 MORPHEUS_MX_SNAC_WK_MAX=$2 timeout -k 10 200 python3 scripts/bench_snac.py --cases 1x1,4x1,7x1,7x4 > $OUT/w$1_k$2.log 2>&1 || exit $?
  echo "waves $1 wk_max $2: $(grep N $OUT/w$1_k$2.log | tr '\n' ' ')"
done
MORPHEUS_MX_SNAC_WAVES=4096 MORPHEUS_MX_SNAC_WK_MAX=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_snac.py > $OUT/tests.log 2>&1; tail -1 $OUT/tests.log
