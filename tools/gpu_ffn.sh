# FFN-backward fusion check: kernel test, micro-bench, step-level tests that run it, bench line.
#   bash tools/gpu_ffn.sh TAG
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-ffn}
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT tests/test_kernels_gpu.py -k ffn > gpurun_out/${TAG}_ffn_test.log 2>&1 || { echo FFN_TEST_FAILED; tail -30 gpurun_out/${TAG}_ffn_test.log; exit 1; }
tail -2 gpurun_out/${TAG}_ffn_test.log
timeout -k 10 200 python -u tools/ffn_bench.py > gpurun_out/${TAG}_ffn_bench.log 2>&1 || { echo FFN_BENCH_FAILED; tail -20 gpurun_out/${TAG}_ffn_bench.log; exit 1; }
cat gpurun_out/${TAG}_ffn_bench.log
if [ -n "$QUICK" ]; then echo FFN_DONE; exit 0; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
S2H_FFN_FUSE=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/${TAG}_bench_nofuse.log 2>&1 || { echo BENCH0_FAILED; tail -20 gpurun_out/${TAG}_bench_nofuse.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench_nofuse.log | cut -c1-300
timeout -k 10 600 $PT tests/test_training_step_gpu.py tests/test_determinism_gpu.py tests/test_graph_gpu.py > gpurun_out/${TAG}_step_tests.log 2>&1 || { echo STEP_TESTS_FAILED; tail -40 gpurun_out/${TAG}_step_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_step_tests.log
echo FFN_DONE
