# Engine session: parity tests of the persistent one-row engine, step A/B against the
# per-kernel graph, and the engine's phase timeline.  Each GPU step has its own time limit;
# a fault / abort / timeout ends the session (nothing further runs on the GPU).
set -u
OUT=${OUT:-gpurun_out/engine}
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -12 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step tests 500 python -u -m pytest ${TESTS:-tests/test_gpu_engine_b1.py} -m gpu -v -p no:cacheprovider -x --timeout 170 --timeout-method thread
[ -z "${TL1:-}" ] || step tl1 200 python -u scripts/engine_timeline.py $TL1
[ -z "${TL2:-}" ] || step tl2 200 python -u scripts/engine_timeline.py $TL2
[ -z "${AB1:-}" ] || step ab1 400 python -u scripts/ab_decode.py $AB1
[ -z "${AB2:-}" ] || step ab2 400 python -u scripts/ab_decode.py $AB2
exit 0
