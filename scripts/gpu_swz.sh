set -u
mkdir -p gpurun_out/swz
timeout -k 10 300 python scripts/bench_rows.py --rows 8,32 --profile-rows 0 --options rows_gen=8 > gpurun_out/swz/plain.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_rows.py --rows 8,32 --profile-rows 0 --options rows_gen=8,rows_dbg=1 > gpurun_out/swz/swz.log 2>&1 || exit $?
tail -n 3 gpurun_out/swz/*.log
