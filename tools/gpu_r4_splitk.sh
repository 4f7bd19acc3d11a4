# round 4: split-major XCD order of split-K weight gradients -- kernel tests, per-shape timing, step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -v -x -k "wgrad or every_tiling or linear_fwd_dgrad" --timeout 120 --timeout-method thread > gpurun_out/r4_splitk_tests.log 2>&1 || { tail -30 gpurun_out/r4_splitk_tests.log; exit 1; }
tail -1 gpurun_out/r4_splitk_tests.log
timeout -k 10 300 python -u tools/splitk_order_bench.py > gpurun_out/r4_splitk_bench.log 2>&1 || { tail -20 gpurun_out/r4_splitk_bench.log; exit 1; }
cat gpurun_out/r4_splitk_bench.log
for r in 1 2; do
  for v in 0 4096; do
    S2H_GEMM_CFG=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_skab_$v$r.log 2> gpurun_out/r4_skab_$v$r.err || { tail -5 gpurun_out/r4_skab_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_skab_$v$r.log'));print('S2H_GEMM_CFG=$v', d['value'], d['ms_per_step'])"
  done
done
