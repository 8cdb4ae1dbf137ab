#!/bin/bash
# One GPU-box session: selected parity tests, a bench run and a rocprofv3 kernel-stats pass.
# Each GPU step has its own time limit; a fault / abort / timeout ends the script.
set -u
OUT=${OUT:-gpurun_out/run}
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
if [ -n "${TESTS:-}" ]; then
  step tests 900 python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider -x --timeout 170 --timeout-method thread
fi
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 900 python bench.py ${BENCH_ARGS:-}
if [ "${SKIP_PROF:-0}" != 1 ]; then
  step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-}
  find "$OUT/prof" -name '*kernel_trace.csv' -delete
  find "$OUT/prof" -name '*.db' -delete
fi
[ -z "${EXTRA:-}" ] || step extra 600 bash -c "$EXTRA"
exit 0
