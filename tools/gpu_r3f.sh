# GEMM tiling rules round: GEMM tests, tiny-M and weight-gradient sweeps, whole-step A/B vs build_ab/A
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread \
  -k "gemm or linear or wgrad or bmm" > gpurun_out/r3f_tests.log 2>&1 || { tail -40 gpurun_out/r3f_tests.log; exit 1; }
tail -2 gpurun_out/r3f_tests.log
timeout -k 10 300 python -u tools/gemm_cfg_sweep.py --tiny > gpurun_out/r3f_tiny.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r3f_tiny.log
timeout -k 10 600 python -u tools/gemm_cfg_sweep.py --wgrad > gpurun_out/r3f_wsweep.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r3f_wsweep.log | cut -c1-60
bash tools/ab_bench.sh 2
