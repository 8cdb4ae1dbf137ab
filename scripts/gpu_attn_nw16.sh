# Multi-row attention in 16-wave blocks (option att_nw_batch=16: one chunk per wave) vs the
# 8-wave default, decode step at L = 600 and 1200, plus the attention kernels' stats.
set -u
OUT=gpurun_out/${TAG:-attn_nw16}
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local t=$1; shift
  timeout -k 10 120 python3 scripts/trace_step.py "$@" > $OUT/$t.log 2>&1 || exit $?
  grep ms/step $OUT/$t.log
}
run r32 --rows 32
run r32_nw16 --rows 32 --opt att_nw_batch=16
run r8f --rows 8 --fp8
run r8f_nw16 --rows 8 --fp8 --opt att_nw_batch=16
run r32_1200 --rows 32 --pos 1200
run r32_1200_nw16 --rows 32 --pos 1200 --opt att_nw_batch=16
timeout -k 10 200 python -u -m pytest -x -q --timeout 170 --timeout-method thread -p no:cacheprovider tests/test_gpu_llm.py -k "batched or rows" > $OUT/tests.log 2>&1; tail -2 $OUT/tests.log
