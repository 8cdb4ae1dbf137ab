# GPU parity tests in one process, verbose with a per-test timeout (a hang names its test).
set -u
OUT=gpurun_out/${TAG:-tests}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 ${SECS:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider -x \
  --timeout ${TEST_TIMEOUT:-170} --timeout-method thread ${PYTEST_ARGS:-} > $OUT/tests.log 2>&1; rc=$?
tail -25 $OUT/tests.log
exit $rc
