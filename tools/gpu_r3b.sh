# round-3 attention scheduling iteration: attention / V-fold / frame-tape tests, then per-kernel
# A/B against build_ab/A (flash forward + backward on the step's shapes, Hiera backward, V-fold
# backward) and the whole step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_vfold_gpu.py tests/test_kernels_gpu.py tests/test_frametape_gpu.py -x -q \
  --timeout 150 --timeout-method thread -k "vfold or flash or attention or attn or frame" \
  > gpurun_out/r3b_tests.log 2>&1 || { tail -40 gpurun_out/r3b_tests.log; exit 1; }
tail -3 gpurun_out/r3b_tests.log
for L in A B; do
  if [ $L = A ]; then export S2H_LIB_PATH=build_ab/A/libsam2hip.so; else unset S2H_LIB_PATH; fi
  timeout -k 10 200 python -u tools/attn_ab.py --iters 10 > gpurun_out/r3b_attn$L.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/hiera_attn_ab.py > gpurun_out/r3b_hiera$L.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/vfold_ab.py --rounds 2 > gpurun_out/r3b_vfold$L.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/r3b_attn$L.log gpurun_out/r3b_hiera$L.log gpurun_out/r3b_vfold$L.log
done
unset S2H_LIB_PATH
bash tools/ab_bench.sh 2
timeout -k 10 300 python -u bench.py --kernel-table --cpu-baseline 0 --steps 5 --warmup 2 > gpurun_out/r3b_ktable.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3b_prof_lib -o lib -- python3 $GRAFT_REPO_ROOT/tools/gemm_vs_lib.py > $GRAFT_REPO_ROOT/gpurun_out/r3b_prof_lib.log 2>&1 || exit 1
