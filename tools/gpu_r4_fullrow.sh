set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "linear_add_ln or every_tiling" --timeout 200 --timeout-method thread > gpurun_out/r4_fullrow_tests.log 2>&1 || { tail -30 gpurun_out/r4_fullrow_tests.log; exit 1; }
tail -2 gpurun_out/r4_fullrow_tests.log
timeout -k 10 300 python -u tools/fullrow_bench.py > gpurun_out/r4_fullrow.log 2>&1 || { tail -20 gpurun_out/r4_fullrow.log; exit 1; }
cat gpurun_out/r4_fullrow.log
