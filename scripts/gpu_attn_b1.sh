# One-row attention shape (waves per block x chunks per wave -> split length) vs the auto
# choice (4 x 1: 128-position splits up to L 1024), decode step ms at three context lengths.
set -u
OUT=gpurun_out/${TAG:-attn_b1}
mkdir -p $OUT
export TMPDIR=/tmp
for pos in 300 600 1000; do
  for o in "" "--opt att_nw=8 --opt att_cpw=1" "--opt att_cpw=2" "--opt att_nw=8 --opt att_cpw=2"; do
    timeout -k 10 120 python3 scripts/trace_step.py --rows 1 --pos $pos --steps 50 $o >> $OUT/steps.log 2>&1 || exit $?
  done
done
grep ms/step $OUT/steps.log
