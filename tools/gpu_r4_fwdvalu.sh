# round 4: flash forward VALU trims (SGPR-based LDS-DMA addressing, integer keep masks, permlane
# reductions, 32-bit hash inputs) -- attention tests, dropout-cost microbench (both query-set forms)
# and step A/B against build_ab/A (HEAD)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_vfold_gpu.py tests/test_frametape_gpu.py -v -x -k "flash or attention or keep or vfold or dropout or query_sets" --timeout 150 --timeout-method thread > gpurun_out/r4_fv_tests.log 2>&1 || { tail -40 gpurun_out/r4_fv_tests.log; exit 1; }
tail -1 gpurun_out/r4_fv_tests.log
S2H_LIB_PATH=build_ab/A/libsam2hip.so timeout -k 10 200 python -u tools/flash_fwd_drop.py > gpurun_out/r4_fv_ffdA.log 2>&1 || { tail -20 gpurun_out/r4_fv_ffdA.log; exit 1; }
S2H_FLASH_QS=17 timeout -k 10 200 python -u tools/flash_fwd_drop.py > gpurun_out/r4_fv_ffdB1.log 2>&1 || { tail -20 gpurun_out/r4_fv_ffdB1.log; exit 1; }
S2H_FLASH_QS=34 timeout -k 10 200 python -u tools/flash_fwd_drop.py > gpurun_out/r4_fv_ffdB2.log 2>&1 || { tail -20 gpurun_out/r4_fv_ffdB2.log; exit 1; }
for f in A B1 B2; do echo $f; grep us/launch gpurun_out/r4_fv_ffd$f.log; done
bash tools/ab_bench.sh 2
