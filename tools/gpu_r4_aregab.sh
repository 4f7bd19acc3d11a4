# round 4: short-K A-in-registers routing -- parity subset, step A/B (S2H_GEMM_AREG 1 / 0)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_training_step_gpu.py -v -x -k "areg or every_tiling or linear or not kernels_gpu" --timeout 150 --timeout-method thread > gpurun_out/r4_aregab_tests.log 2>&1 || { tail -30 gpurun_out/r4_aregab_tests.log; exit 1; }
tail -1 gpurun_out/r4_aregab_tests.log
for r in 1 2; do
  for v in 1 0; do
    S2H_GEMM_AREG=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_aregab_$v$r.log 2> gpurun_out/r4_aregab_$v$r.err || { tail -5 gpurun_out/r4_aregab_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_aregab_$v$r.log'));print('S2H_GEMM_AREG=$v', d['value'], d['ms_per_step'])"
  done
done
