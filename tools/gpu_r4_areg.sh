# round 4: short-K GEMM with A in registers -- kernel tests, per-shape timing
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -v -x -k "areg or every_tiling" --timeout 120 --timeout-method thread > gpurun_out/r4_areg_tests.log 2>&1 || { tail -30 gpurun_out/r4_areg_tests.log; exit 1; }
tail -1 gpurun_out/r4_areg_tests.log
timeout -k 10 300 python -u tools/areg_bench.py > gpurun_out/r4_areg_bench.log 2>&1 || { tail -20 gpurun_out/r4_areg_bench.log; exit 1; }
cat gpurun_out/r4_areg_bench.log
