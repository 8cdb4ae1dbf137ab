#!/bin/bash
# GPU session: parity tests, smoke, then B=1 decode-step kernel traces (bf16, fp8) with gaps.
# Each GPU step has its own limit; a fault / abort / timeout ends the script.
set -u
OUT=${OUT:-gpurun_out/traces}
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -4 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step tests ${TEST_SECS:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for v in ${TRACES:-}; do   # e.g. TRACES="bf16 fp8"
  flag=""; [ "$v" = fp8 ] && flag="--fp8"
  step trace_$v 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$v" -o run -- python3 scripts/trace_step.py $flag ${TRACE_ARGS:-}
  f=$(find "$OUT/trace_$v" -name '*kernel_trace.csv' | head -1)
  [ -n "$f" ] && python3 scripts/step_gaps.py "$f" 10 ${MARKER:-commit_kernel} > "$OUT/gaps_$v.txt" && cat "$OUT/gaps_$v.txt" | head -20
  find "$OUT/trace_$v" -name '*.csv' -size +5M -delete
done
[ "${SKIP_BENCH:-1}" = 1 ] || step bench 900 python bench.py ${BENCH_ARGS:-}
exit 0
