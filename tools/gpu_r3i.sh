# loss kernels: tests, then the whole-step A/B against build_ab/A
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_training_step_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3i_tests.log 2>&1 || { tail -40 gpurun_out/r3i_tests.log; exit 1; }
tail -2 gpurun_out/r3i_tests.log
bash tools/ab_bench.sh 2
