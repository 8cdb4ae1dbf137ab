set -u
OUT=gpurun_out/ab_head; mkdir -p $OUT
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --variants base,hmt2 --pos 600 --rounds 2 > $OUT/r8.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_decode.py --rows 8 --fp8 --variants base,hmt2 --pos 600 --rounds 2 > $OUT/r8fp8.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_decode.py --rows 32 --variants base,hmt2 --pos 600 --rounds 2 > $OUT/r32.log 2>&1
rc=$?; grep -h -v amdgpu $OUT/*.log | grep -v round; exit $rc
