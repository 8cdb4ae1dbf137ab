set -u
OUT=gpurun_out/${TAG:-ntmax}
mkdir -p $OUT
export TMPDIR=/tmp
for nt in ${NTS:-0 1}; do :; done; for mt in 0 1; do nt=mt2_$mt
  timeout -k 10 300 python3 -u scripts/bench_rows.py --rows 32 --profile-rows 32 --options rows_mt2=$mt > $OUT/nt$nt.log 2>&1 || exit $?
  echo "== rows_nt_max $nt"; grep -v amdgpu.ids $OUT/nt$nt.log
done
