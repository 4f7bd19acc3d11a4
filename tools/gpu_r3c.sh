# GEMM tiling sweep after the translation-unit split: every tiling's correctness, then the
# config sweep on the step's shapes (hipBLASLt alongside)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread \
  -k "gemm or linear or wgrad or bmm" > gpurun_out/r3c_tests.log 2>&1 || { tail -40 gpurun_out/r3c_tests.log; exit 1; }
tail -2 gpurun_out/r3c_tests.log
timeout -k 10 400 python -u tools/gemm_cfg_sweep.py > gpurun_out/r3c_sweep.log 2>&1 || { tail -20 gpurun_out/r3c_sweep.log; exit 1; }
grep -v amdgpu gpurun_out/r3c_sweep.log
