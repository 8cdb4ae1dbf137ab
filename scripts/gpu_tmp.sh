set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ab32g
timeout -k 10 600 python -m pytest tests/test_gpu_llm.py -q -p no:cacheprovider -x > gpurun_out/ab32g/tests.log 2>&1; rc=$?
tail -2 gpurun_out/ab32g/tests.log
case $rc in 124|134|137|139) exit $rc;; esac
OUT=gpurun_out/ab32g bash scripts/gpu_ab32.sh
