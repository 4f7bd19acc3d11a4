# round-3 kernel iteration: GEMM / flash / V-fold tests, V-fold dK A/B, GEMM shapes A/B
# (A = build_ab/A/libsam2hip.so), whole-step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_vfold_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "vfold or gemm or linear or wgrad or bmm or flash or attention" \
  > gpurun_out/r3a_tests.log 2>&1 || { tail -40 gpurun_out/r3a_tests.log; exit 1; }
tail -3 gpurun_out/r3a_tests.log
timeout -k 10 200 python -u tools/vfold_ab.py > gpurun_out/r3a_vfold.log 2>&1 || { tail -20 gpurun_out/r3a_vfold.log; exit 1; }
cat gpurun_out/r3a_vfold.log
S2H_LIB_PATH=build_ab/A/libsam2hip.so timeout -k 10 300 python -u tools/gemm_vs_lib.py > gpurun_out/r3a_gemmA.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_vs_lib.py > gpurun_out/r3a_gemmB.log 2>&1 || exit 1
paste gpurun_out/r3a_gemmA.log gpurun_out/r3a_gemmB.log | cut -c1-140
bash tools/ab_bench.sh 2
