# batched bank / gradient-packing copies: their tests + the step suites that run through them, then
# an in-call A/B of the whole step (S2H_COPY_BATCH=0: one Tensor.copy_ per pair)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_copy_segments.py tests/test_frametape_gpu.py tests/test_training_step_gpu.py tests/test_graph_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_v23_copyseg_tests.log 2>&1 || { tail -30 gpurun_out/r04_v23_copyseg_tests.log; exit 1; }
tail -2 gpurun_out/r04_v23_copyseg_tests.log
VAR=S2H_COPY_BATCH A=0 B=1 STEPS=30 bash tools/gpu_ab_env.sh 2>&1 | tee gpurun_out/r04_v23_copyseg_ab.log
