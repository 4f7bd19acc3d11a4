# round-6: run chosen GPU test files (args) under one pytest process, log to gpurun_out/TAG_tests.log
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -40
exit $rc
