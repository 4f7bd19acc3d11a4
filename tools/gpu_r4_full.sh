# full GPU suite (all failures reported), smoke, bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r4}
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?
tail -25 gpurun_out/${T}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.log
exit $rc
