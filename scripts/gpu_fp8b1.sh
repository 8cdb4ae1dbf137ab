set -u
mkdir -p gpurun_out/f8b1
timeout -k 10 400 python scripts/ab_decode.py --fp8 --rounds 2 --pos 600 --variants base,rpw_gu4,rpw_down2,gu4_down2,wpb8,rpw_o2 > gpurun_out/f8b1/ab.log 2>&1 || exit $?
tail -7 gpurun_out/f8b1/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f8b1/prof -o run -- python3 scripts/ab_decode.py --fp8 --rounds 1 --pos 600 --variants base > gpurun_out/f8b1/prof.log 2>&1 || exit $?
find gpurun_out/f8b1/prof -name '*kernel_trace.csv' -delete; find gpurun_out/f8b1/prof -name '*.db' -delete
