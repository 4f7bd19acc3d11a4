# round 4: fused projection + residual + LayerNorm (s2h_linear_add_ln) -- kernel / model parity, timing, step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_vfold_gpu.py tests/test_frametape_gpu.py tests/test_parity_gpu.py tests/test_training_step_gpu.py -q -x -k "linear_add_ln or every_tiling or not kernels_gpu" --timeout 200 --timeout-method thread > gpurun_out/r4_ln_tests.log 2>&1 || { tail -40 gpurun_out/r4_ln_tests.log; exit 1; }
tail -2 gpurun_out/r4_ln_tests.log
timeout -k 10 300 python -u tools/fullrow_bench.py > gpurun_out/r4_fullrow.log 2>&1 || { tail -20 gpurun_out/r4_fullrow.log; exit 1; }
cat gpurun_out/r4_fullrow.log
for r in 1 2; do
  for v in 1 0; do
    S2H_LINEAR_LN=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_lnab_$v$r.log 2> gpurun_out/r4_lnab_$v$r.err || { tail -5 gpurun_out/r4_lnab_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_lnab_$v$r.log'));print('LINEAR_LN=$v', d['value'], d['ms_per_step'])"
  done
done
