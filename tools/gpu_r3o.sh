# persistent short-K GEMM: bitwise / tiling tests, then the short-K forward GEMM breakdown (cold and hot)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "wave_grid or (every_tiling and (20 or 21 or 22 or 23 or 24))" > gpurun_out/r3o_tests.log 2>&1 || { tail -30 gpurun_out/r3o_tests.log; exit 1; }
tail -2 gpurun_out/r3o_tests.log
timeout -k 10 500 python -u tools/gemm_breakdown.py > gpurun_out/r3o_cold.log 2>&1 || { tail -20 gpurun_out/r3o_cold.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3o_cold.log
timeout -k 10 300 python -u tools/gemm_breakdown.py --hot --ablate 0 > gpurun_out/r3o_hot.log 2>&1 || { tail -20 gpurun_out/r3o_hot.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3o_hot.log
