#!/bin/bash
# One GPU-box session for a kernel A/B: optional parity tests under engine-option overrides
# (MORPHEUS_MX_OPT_<key>=<v>, set by the caller), then scripts/ab_decode.py runs (AB1..AB6:
# argument strings).  Each GPU step has its own time limit; a fault / abort / timeout ends it.
set -u
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -12 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
if [ -n "${TESTS:-}" ]; then
  step tests ${TEST_SECS:-900} python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider -x --timeout 170 --timeout-method thread -k "${PYTEST_K:-}"
fi
[ -z "${AB1:-}" ] || step ab1 400 python -u scripts/ab_decode.py $AB1
[ -z "${AB2:-}" ] || step ab2 400 python -u scripts/ab_decode.py $AB2
[ -z "${AB3:-}" ] || step ab3 400 python -u scripts/ab_decode.py $AB3
[ -z "${AB4:-}" ] || step ab4 400 python -u scripts/ab_decode.py $AB4
[ -z "${AB5:-}" ] || step ab5 400 python -u scripts/ab_decode.py $AB5
[ -z "${AB6:-}" ] || step ab6 400 python -u scripts/ab_decode.py $AB6
exit 0
