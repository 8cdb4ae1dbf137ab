set -u
OUT=gpurun_out/${TAG:-f8pw}
mkdir -p $OUT
export TMPDIR=/tmp
for pw in ${PWS:-2 3}; do
  timeout -k 10 300 python3 -u scripts/bench_rows.py --rows 8 --profile-rows 8 --fp8 --options rows_pw_f8=$pw > $OUT/f8_pw$pw.log 2>&1 || exit $?
  echo "== fp8 rows_pw_f8 $pw"; grep -v amdgpu.ids $OUT/f8_pw$pw.log
done
