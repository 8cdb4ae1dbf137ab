#!/bin/bash
# round 6: Infinity-Cache bound of the decode GEMVs; multi-row block timelines before (seam) /
# after (atomics + qkv partials); the multi-row PMC records of the seam-free path
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r06_n; mkdir -p $OUT
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log"
  [ $rc = 0 ] || exit $rc
}
step mall_bf16 300 python3 scripts/mall_bound.py --rows 1,8
step mall_fp8 300 python3 scripts/mall_bound.py --rows 1,8 --fp8
TL=project_morpheus_amd/libmorpheus_mx_trace.so
step blk_after 300 env MORPHEUS_MX_LIB=$TL python3 scripts/rows_block_trace.py --rows 8,32 --kinds qkv,o_proj,gate_up,down
step blk_before 300 env MORPHEUS_MX_LIB=$TL python3 scripts/rows_block_trace.py --rows 8,32 --kinds qkv,o_proj,gate_up,down --options rows_atomic=0,rows_qkv_parts=0
step blk_after_fp8 300 env MORPHEUS_MX_LIB=$TL python3 scripts/rows_block_trace.py --rows 8 --fp8 --kinds qkv,o_proj,gate_up,down
step blk_before_fp8 300 env MORPHEUS_MX_LIB=$TL python3 scripts/rows_block_trace.py --rows 8 --fp8 --kinds qkv,o_proj,gate_up,down --options rows_atomic=0,rows_qkv_parts=0
OUT=$OUT/pmc bash scripts/gpu_pmc_rows_kinds.sh > $OUT/pmc.log 2>&1 || { echo "pmc FAILED"; tail -5 $OUT/pmc.log; exit 1; }
tail -5 $OUT/pmc.log
