# round 4: flash forward with two 16-query sets per wave (+ permlane reductions, 32-bit hash inputs) --
# attention tests, dropout-cost microbench and step A/B against build_ab/A (HEAD)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vfold_gpu.py tests/test_frametape_gpu.py -v -x -k "flash or attention or keep or vfold or dropout or query_sets" --timeout 150 --timeout-method thread > gpurun_out/r4_qs_tests.log 2>&1 || { tail -40 gpurun_out/r4_qs_tests.log; exit 1; }
tail -1 gpurun_out/r4_qs_tests.log
S2H_LIB_PATH=build_ab/A/libsam2hip.so timeout -k 10 200 python -u tools/flash_fwd_drop.py > gpurun_out/r4_qs_ffdA.log 2>&1 || { tail -20 gpurun_out/r4_qs_ffdA.log; exit 1; }
timeout -k 10 200 python -u tools/flash_fwd_drop.py > gpurun_out/r4_qs_ffdB.log 2>&1 || { tail -20 gpurun_out/r4_qs_ffdB.log; exit 1; }
echo A; grep us/launch gpurun_out/r4_qs_ffdA.log; echo B; grep us/launch gpurun_out/r4_qs_ffdB.log
bash tools/ab_bench.sh 2
