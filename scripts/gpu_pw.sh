mkdir -p gpurun_out/pw
for pw in 1 2; do
  timeout -k 10 300 python scripts/bench_rows.py --rows 8,32,64 --profile-rows 32 --options rows_pw=$pw,rows_pw_f8=$pw > gpurun_out/pw/pw$pw.log 2>&1 || exit $?
done
timeout -k 10 300 python scripts/bench_rows.py --rows 8,32 --profile-rows 8 --fp8 --options rows_pw_f8=2 > gpurun_out/pw/f8_pw2.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_rows.py --rows 8,32 --profile-rows 8 --fp8 --options rows_pw_f8=4 > gpurun_out/pw/f8_pw4.log 2>&1
