# kernel + parity + graph tests on the current build, then the whole-step A/B against build_ab/A
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_vfold_gpu.py tests/test_parity_gpu.py \
  tests/test_graph_gpu.py tests/test_frametape_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r3d_tests.log 2>&1 || { tail -40 gpurun_out/r3d_tests.log; exit 1; }
tail -2 gpurun_out/r3d_tests.log
bash tools/ab_bench.sh 2
timeout -k 10 300 python -u bench.py --kernel-table --cpu-baseline 0 --steps 5 --warmup 2 > gpurun_out/r3d_ktable.log 2>&1 || exit 1
grep "attn_.*d16\|gemm .*13312x2048x256\|gemm .*93184x256x2048" gpurun_out/r3d_ktable.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3d_trace -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r3d_trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/trace_gaps.py $(find gpurun_out/r3d_trace -name "*.db" | head -1) --steps 3
