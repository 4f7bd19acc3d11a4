# kernel tests of the GEMM paths + parity, then the default bench (run via gpurun)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_mx8_gpu.py tests/test_parity_gpu.py tests/test_frametape_gpu.py -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/qb_tests.log 2>&1
rc=$?
tail -3 gpurun_out/qb_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/qb_tests.log; exit $rc; }
timeout -k 10 400 python -u bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/qb_bench.log 2> gpurun_out/qb_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/qb_bench.err; exit 1; }
cat gpurun_out/qb_bench.log
