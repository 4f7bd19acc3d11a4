# round 4: flash forward softmax reductions on v_permlane16/32_swap + 32-bit dropout hash inputs --
# attention tests, dropout-cost microbench and step A/B against build_ab/A (HEAD)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vfold_gpu.py tests/test_frametape_gpu.py -v -x -k "flash or attention or keep or vfold or dropout" --timeout 150 --timeout-method thread > gpurun_out/r4_pl_tests.log 2>&1 || { tail -40 gpurun_out/r4_pl_tests.log; exit 1; }
tail -1 gpurun_out/r4_pl_tests.log
S2H_LIB_PATH=build_ab/A/libsam2hip.so timeout -k 10 200 python -u tools/flash_fwd_drop.py > gpurun_out/r4_pl_ffdA.log 2>&1 || { tail -20 gpurun_out/r4_pl_ffdA.log; exit 1; }
timeout -k 10 200 python -u tools/flash_fwd_drop.py > gpurun_out/r4_pl_ffdB.log 2>&1 || { tail -20 gpurun_out/r4_pl_ffdB.log; exit 1; }
echo A; grep us/launch gpurun_out/r4_pl_ffdA.log; echo B; grep us/launch gpurun_out/r4_pl_ffdB.log
bash tools/ab_bench.sh 2
