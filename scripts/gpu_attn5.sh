set -u
OUT=gpurun_out/${TAG:-attn5}
mkdir -p $OUT
export TMPDIR=/tmp
A="timeout -k 10 200 python3 -u scripts/pmc_attn.py --rows 1 --lens 100,300,600,900,1200"
{ for nw in 4 8; do for c in 1 2 4; do $A --nw $nw --cpw $c || exit 1; done; done; } > $OUT/sweep.log 2>&1 || exit $?
grep '"rows"' $OUT/sweep.log
