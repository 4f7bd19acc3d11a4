# two-wave dK/dV kernel for head dim 256: attention tests, kernel A/B (variant 3 = old), step A/B vs build_ab/A
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_vfold_gpu.py tests/test_kernels_gpu.py tests/test_frametape_gpu.py tests/test_graph_gpu.py -x -q \
  --timeout 200 --timeout-method thread -k "vfold or flash or attention or attn or frame or graph" \
  > gpurun_out/r3j_tests.log 2>&1 || { tail -40 gpurun_out/r3j_tests.log; exit 1; }
tail -2 gpurun_out/r3j_tests.log
timeout -k 10 200 python -u tools/attn_ab.py --iters 10 --variants > gpurun_out/r3j_attn.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/vfold_ab.py --rounds 2 > gpurun_out/r3j_vfold.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r3j_attn.log gpurun_out/r3j_vfold.log
bash tools/ab_bench.sh 2
