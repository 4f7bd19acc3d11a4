# one GPU call: a focused pytest selection (TESTS, -k K) then the default bench with the kernel
# table (BENCH=0 skips it).   TESTS="tests/a.py tests/b.py" K="expr" bash tools/gpu_focus.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} ${K:+-k "$K"} -m gpu -v -rf --timeout 200 --timeout-method thread > gpurun_out/focus_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/focus_tests.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python -u bench.py --cpu-baseline 0 --kernel-table ${BENCH_ARGS} > gpurun_out/focus_bench.log 2> gpurun_out/focus_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/focus_bench.err; exit 1; }
  cat gpurun_out/focus_bench.log
  head -40 gpurun_out/focus_bench.err
fi
exit $rc
