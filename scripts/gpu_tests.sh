set -u
OUT=gpurun_out/${TAG:-tests}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider -x ${PYTEST_ARGS:-} > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log
exit $rc
