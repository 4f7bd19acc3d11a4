# round 4: flash backward (dQ, V-fold dK) stage loads on SGPR row bases with precomputed lane offsets
# -- attention tests, V-fold backward microbench and step A/B against build_ab/A (HEAD)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vfold_gpu.py tests/test_frametape_gpu.py -v -x -k "flash or attention or keep or vfold or dropout or query_sets" --timeout 150 --timeout-method thread > gpurun_out/r4_bd_tests.log 2>&1 || { tail -40 gpurun_out/r4_bd_tests.log; exit 1; }
tail -1 gpurun_out/r4_bd_tests.log
S2H_LIB_PATH=build_ab/A/libsam2hip.so timeout -k 10 200 python -u tools/vfold_ab.py > gpurun_out/r4_bd_vfA.log 2>&1 || { tail -20 gpurun_out/r4_bd_vfA.log; exit 1; }
timeout -k 10 200 python -u tools/vfold_ab.py > gpurun_out/r4_bd_vfB.log 2>&1 || { tail -20 gpurun_out/r4_bd_vfB.log; exit 1; }
echo A; grep variant gpurun_out/r4_bd_vfA.log; echo B; grep variant gpurun_out/r4_bd_vfB.log
bash tools/ab_bench.sh 2
