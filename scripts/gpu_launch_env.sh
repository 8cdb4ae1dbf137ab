#!/bin/bash
# Graph node cost and the one-row decode step under HIP runtime knobs (launch-latency study).
set -u
OUT=${OUT:-gpurun_out/launch_env}
mkdir -p "$OUT"
run() {
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  cat "$OUT/$name.log" | tail -12
  case $rc in 0) return 0;; *) exit $rc;; esac
}
run floor_base 120 scripts/micro/launch_floor
HIP_FORCE_DEV_KERNARG=1 run floor_devkarg1 120 scripts/micro/launch_floor
HIP_FORCE_DEV_KERNARG=0 run floor_devkarg0 120 scripts/micro/launch_floor
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run floor_nocapture 120 scripts/micro/launch_floor
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 run floor_capture 120 scripts/micro/launch_floor
run step_base 300 python -u scripts/ab_decode.py --variants base --pos 600 --rounds 2
HIP_FORCE_DEV_KERNARG=1 run step_devkarg1 300 python -u scripts/ab_decode.py --variants base --pos 600 --rounds 2
HIP_FORCE_DEV_KERNARG=0 run step_devkarg0 300 python -u scripts/ab_decode.py --variants base --pos 600 --rounds 2
exit 0
