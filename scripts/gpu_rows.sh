#!/bin/bash
# Multi-row decode A/B session: parity tests of the multi-row paths, step traces at 8 / 32 /
# 64 rows, then the batched bench sections.
set -u
OUT=${OUT:-gpurun_out/rows}
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
if [ "${ALL_TESTS:-0}" = 1 ]; then
  step tests 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread
elif [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests 600 python -u -m pytest tests/test_gpu_llm.py tests/test_gpu_fp8.py tests/test_gpu_batching.py -m gpu -k "batched or rows or fp8 or batch" -v -p no:cacheprovider --timeout 170 --timeout-method thread
fi
step r1 200 python scripts/trace_step.py --rows 1 --steps 50
step r32 200 python scripts/trace_step.py --rows 32 --steps 20
step r64 200 python scripts/trace_step.py --rows 64 --steps 20
step r8f8 200 python scripts/trace_step.py --rows 8 --fp8 --steps 20
step r16 200 python scripts/trace_step.py --rows 16 --steps 20
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py --no-http --no-cpu-baseline --steps 1 --warmup 1
grep -h "ms/step" $OUT/r*.log
exit 0
