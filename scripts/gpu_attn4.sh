set -u
OUT=gpurun_out/${TAG:-attn4}
mkdir -p $OUT
export TMPDIR=/tmp
A="timeout -k 10 200 python3 -u scripts/pmc_attn.py"
{ for R in 4 8 16; do
    $A --rows $R --lens 300,600,1200 --nw 8 --cpw 1 && $A --rows $R --lens 300,600,1200 --nw 8 --cpw 2 \
    && $A --rows $R --lens 300,600,1200 --nw 4 --cpw 1 && $A --rows $R --lens 300,600,1200 --nw 4 --cpw 2 || exit 1
  done; } > $OUT/sweep.log 2>&1 || exit $?
grep '"rows"' $OUT/sweep.log
