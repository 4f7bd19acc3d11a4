# fused V-fold + output projection: V-fold / parity / graph / frame-tape / training-step tests, step A/B by env switch
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_vfold_gpu.py tests/test_parity_gpu.py tests/test_graph_gpu.py \
  tests/test_frametape_gpu.py tests/test_training_step_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3k_tests.log 2>&1 || { tail -40 gpurun_out/r3k_tests.log; exit 1; }
tail -2 gpurun_out/r3k_tests.log
VAR=S2H_VFOLD_OUT A=0 B=1 bash tools/gpu_ab_env.sh
