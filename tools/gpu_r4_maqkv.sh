# round 4: memory-attention layer-0 norm1 + q/k/v once per frame -- tape equivalence, parity, step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_frametape_gpu.py tests/test_parity_gpu.py tests/test_training_step_gpu.py tests/test_determinism_gpu.py tests/test_graph_gpu.py tests/test_predictor_gpu.py tests/test_eval.py -v -s -x -k "ma_shared_qkv or not kernels_gpu" --timeout 150 --timeout-method thread > gpurun_out/r4_maqkv_tests.log 2>&1 || { tail -40 gpurun_out/r4_maqkv_tests.log; exit 1; }
tail -1 gpurun_out/r4_maqkv_tests.log
grep -h "S2H_MA_SHARED_QKV=1" gpurun_out/r4_maqkv_tests.log || true
for r in 1 2; do
  for v in 1 0; do
    S2H_MA_SHARED_QKV=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_maqkv_$v$r.log 2> gpurun_out/r4_maqkv_$v$r.err || { tail -5 gpurun_out/r4_maqkv_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_maqkv_$v$r.log'));print('S2H_MA_SHARED_QKV=$v', d['value'], d['ms_per_step'])"
  done
done
