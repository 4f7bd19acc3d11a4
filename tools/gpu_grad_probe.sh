# the bf16 8-frame training-step gradient report under several environment switches (diagnostic)
set -o pipefail
mkdir -p gpurun_out
T=tests/test_training_step_gpu.py::test_training_step_bf16_t8_matches_reference_bf16_drift
for e in "X=1" "S2H_CONVT_DIRECT=0" "S2H_CONVT_DIRECT=0 S2H_HIERA_WIN_STAGE=0 S2H_GRAD_DEFER=0" "S2H_DEC_TOK=0"; do
  echo "== $e"
  env $e timeout -k 10 200 python -u -m pytest -q -s --timeout 150 $T 2>&1 | grep -E "worst gradient|passed|failed" | cut -c1-900
done
exit 0
