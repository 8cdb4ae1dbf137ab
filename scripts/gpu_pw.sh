set -u
OUT=gpurun_out/${TAG:-pw}
mkdir -p $OUT
export TMPDIR=/tmp
for pw in ${PWS:-1 2 3}; do
  timeout -k 10 300 python3 -u scripts/bench_rows.py --rows ${ROWS:-8,32} --profile-rows 0 --options rows_pw=$pw > $OUT/rows_pw$pw.log 2>&1 || exit $?
  echo "== rows_pw $pw"; grep -v amdgpu.ids $OUT/rows_pw$pw.log
done
