#!/bin/bash
# Round check on one GPU box: all parity tests, smoke, the full bench, rocprofv3 kernel stats.
set -u
OUT=${OUT:-gpurun_out/full}
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
[ "${SKIP_TESTS:-0}" = 1 ] || step tests 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 900 python bench.py ${BENCH_ARGS:-}
if [ "${SKIP_PROF:-0}" != 1 ]; then
  step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline
  find "$OUT/prof" -name '*kernel_trace.csv' -delete
  find "$OUT/prof" -name '*.db' -delete
fi
exit 0
