# round 4: fused projection + residual + LayerNorm (s2h_linear_add_ln), LayerNorm backward in the dgrad
# epilogue (s2h_linear_dgrad_ln_bwd) -- kernel / model parity, timing, step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_vfold_gpu.py tests/test_frametape_gpu.py tests/test_parity_gpu.py tests/test_training_step_gpu.py -v -s -x -k "linear_add_ln or linear_dgrad_ln or every_tiling or not kernels_gpu" --timeout 120 --timeout-method thread > gpurun_out/r4_ln_tests.log 2>&1 || { tail -40 gpurun_out/r4_ln_tests.log; exit 1; }
tail -2 gpurun_out/r4_ln_tests.log
grep -h "fused LayerNorm backward" gpurun_out/r4_ln_tests.log || true
timeout -k 10 300 python -u tools/fullrow_bench.py > gpurun_out/r4_fullrow.log 2>&1 || { tail -20 gpurun_out/r4_fullrow.log; exit 1; }
cat gpurun_out/r4_fullrow.log
for r in 1 2; do
  for v in 11 10 00; do
    S2H_LINEAR_LN=${v:0:1} S2H_LN_BWD_FUSE=${v:1:1} timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_lnab_$v$r.log 2> gpurun_out/r4_lnab_$v$r.err || { tail -5 gpurun_out/r4_lnab_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_lnab_$v$r.log'));print('LINEAR_LN,LN_BWD_FUSE=$v', d['value'], d['ms_per_step'])"
  done
done
