#!/bin/bash
# XCD-aware K-range order in the multi-row GEMM: parity tests, step timings, the FETCH_SIZE pass
# of the 32-row projections, then configs[2] with and without decode-row compaction.
set -u
OUT=${OUT:-gpurun_out/xcdrows}
mkdir -p $OUT
export TMPDIR=/tmp
SKIP_BENCH=1 OUT=$OUT bash scripts/gpu_rows.sh || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r32_fetch -o r32_fetch -- python3 scripts/pmc_gemv.py --rows 32 > $OUT/r32_fetch.log 2>&1 || { echo "FAILED fetch"; tail -5 $OUT/r32_fetch.log; exit 1; }
f=$(find $OUT/r32_fetch -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summary.py $f --kernel gemm_rows > $OUT/r32_fetch.summary.json
rm -f $f
cat $OUT/r32_fetch.summary.json
timeout -k 10 600 python3 bench.py --no-http --no-cpu-baseline --steps 1 --warmup 1 --long-read-docs 0 --fp8-batch 0 --compaction-ab > $OUT/bench_compaction.log 2>&1 || { tail -5 $OUT/bench_compaction.log; exit 1; }
grep '^{' $OUT/bench_compaction.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['configs_2_batched'])); print(json.dumps(d.get('configs_2_no_compaction')))"
