# parity + tape tests, then the bench with the per-shape kernel table
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_frametape_gpu.py tests/test_graph_gpu.py tests/test_configs_gpu.py -q -rf --timeout 150 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -8 gpurun_out/quick_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit $rc; fi
timeout -k 10 400 python -u bench.py --kernel-table --cpu-baseline 0 > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
exit $rc
