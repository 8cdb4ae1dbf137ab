set -u
OUT=gpurun_out/${TAG:-target}
mkdir -p $OUT
export TMPDIR=/tmp
for t in ${TARGETS:-384 192 128}; do
  timeout -k 10 300 python3 -u scripts/bench_rows.py --rows ${ROWS:-8,32} --profile-rows 0 --options rows_target=$t > $OUT/rows_t$t.log 2>&1 || exit $?
  echo "== rows_target $t"; grep -v amdgpu.ids $OUT/rows_t$t.log
done
for cpw in ${CPWS:-1 2 4}; do
  timeout -k 10 300 python3 -u scripts/bench_rows.py --rows 32 --profile-rows 32 --options att_cpw_batch=$cpw > $OUT/att_cpw$cpw.log 2>&1 || exit $?
  echo "== att_cpw_batch $cpw"; grep profile_rows $OUT/att_cpw$cpw.log
done
