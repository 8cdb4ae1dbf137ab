# fp8 MFMA multi-row GEMM (option rows_f8m) vs the fp8 -> bf16 path: parity, then the 8-row
# (configs[4] per GPU) and 16-row decode steps, and prefill (16 ids: one batch tile).
set -u
OUT=gpurun_out/${TAG:-f8m}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fp8.py > $OUT/tests.log 2>&1; rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
grep -E "PASS|FAIL|passed|failed" $OUT/tests.log | tail -12
for r in 8 16; do
  for o in 0 1; do
    timeout -k 10 120 python3 scripts/trace_step.py --rows $r --fp8 --opt rows_f8m=$o > $OUT/step_r${r}_f8m$o.log 2>&1 || exit $?
    grep ms/step $OUT/step_r${r}_f8m$o.log
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 scripts/trace_step.py --rows 8 --fp8 --opt rows_f8m=1 > $OUT/kt.log 2>&1 || exit $?
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/stats_r8_f8m1.csv \;
find $OUT/kt -name '*kernel_trace.csv' -delete
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/" + __import__("os").environ.get("TAG", "f8m") + "/stats_r8_f8m1.csv")[0]
for r in csv.DictReader(open(f)):
    if "gemm_rows" in r["Name"] or "attn" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:8.2f} us  x{r["Calls"]:>6}  {r["Name"][:90]}')
PY
