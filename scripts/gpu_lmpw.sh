set -u
OUT=gpurun_out/${TAG:-lmpw}
mkdir -p $OUT
export TMPDIR=/tmp
for pw in 1 2; do
  timeout -k 10 300 python3 -u scripts/bench_rows.py --rows 32 --profile-rows 32 --options rows_pw=$pw > $OUT/pw$pw.log 2>&1 || exit $?
  echo "== rows_pw $pw"; grep profile_rows $OUT/pw$pw.log
done
