# Multi-row attention split policy at L = 600: auto (R = 8: 3 splits of 256 + ticket merge) vs
# forced chunks per wave (3 -> one split of 768, no merge), decode step ms.
set -u
OUT=gpurun_out/${TAG:-attn_rows_ab}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # tag args...
  local t=$1; shift
  timeout -k 10 120 python3 scripts/trace_step.py "$@" > $OUT/$t.log 2>&1 || exit $?
  grep ms/step $OUT/$t.log
}
run r8f_auto --rows 8 --fp8
run r8f_c2 --rows 8 --fp8 --opt att_cpw_batch=2
run r8f_c3 --rows 8 --fp8 --opt att_cpw_batch=3
run r8f_c4 --rows 8 --fp8 --opt att_cpw_batch=4
run r16f_auto --rows 16 --fp8
run r16f_c3 --rows 16 --fp8 --opt att_cpw_batch=3
run r8b_auto --rows 8
run r8b_c3 --rows 8 --opt att_cpw_batch=3
run r8f_auto2 --rows 8 --fp8
