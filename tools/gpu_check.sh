# parity + tape + graph + config tests, the default bench (with the CPU baseline), torch profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_frametape_gpu.py tests/test_graph_gpu.py tests/test_configs_gpu.py -q -rf --timeout 150 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -3 gpurun_out/quick_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit $rc; fi
START=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_default.err; exit 1; }
echo "default bench wall: $(( $(date +%s) - START )) s"
cat gpurun_out/bench_default.log
timeout -k 10 300 python tools/torch_prof.py --rows 5 > gpurun_out/torch_prof.log 2>&1 || echo PROF_FAILED
exit $rc
