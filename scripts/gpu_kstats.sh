#!/bin/bash
# rocprofv3 kernel stats of decode steps under option sets: RUNS="name:opt1=v,opt2=v name2:..."
# (trace_step.py ARGS shared), kstats summaries to $OUT/<name>.txt; traces deleted.
set -u
OUT=${OUT:-gpurun_out/kstats}
mkdir -p "$OUT"
export TMPDIR=/tmp
for run in ${RUNS}; do
  name=${run%%:*}; opts=${run#*:}
  optargs=""
  for kv in ${opts//,/ }; do [ "$kv" = "-" ] || optargs="$optargs --opt $kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- python3 scripts/trace_step.py ${ARGS:-} $optargs > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log"
  case $rc in 0) ;; *) exit $rc;; esac
  f=$(find "$OUT/$name" -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && python3 scripts/kstats.py "$f" 14 > "$OUT/$name.txt" && cat "$OUT/$name.txt"
  find "$OUT/$name" -name '*kernel_trace.csv' -delete
  find "$OUT/$name" -name '*.db' -delete
done
[ -z "${AB1:-}" ] || { timeout -k 10 400 python -u scripts/ab_decode.py $AB1 > "$OUT/ab1.log" 2>&1; echo "== ab1 rc=$?"; tail -6 "$OUT/ab1.log"; }
[ -z "${AB2:-}" ] || { timeout -k 10 400 python -u scripts/ab_decode.py $AB2 > "$OUT/ab2.log" 2>&1; echo "== ab2 rc=$?"; tail -6 "$OUT/ab2.log"; }
exit 0
