# round 4: weight gradients on a second stream (ops.SideWork) -- equivalence tests, step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_frametape_gpu.py tests/test_determinism_gpu.py tests/test_graph_gpu.py -v -s -x -k "not S2H_LINEAR_LN" --timeout 150 --timeout-method thread > gpurun_out/r4_side_tests.log 2>&1 || { tail -40 gpurun_out/r4_side_tests.log; exit 1; }
tail -2 gpurun_out/r4_side_tests.log
grep -h "launches, global\|worst" gpurun_out/r4_side_tests.log || true
for r in 1 2; do
  for v in 1 0; do
    S2H_WGRAD_STREAM=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_sideab_$v$r.log 2> gpurun_out/r4_sideab_$v$r.err || { tail -5 gpurun_out/r4_sideab_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_sideab_$v$r.log'));print('WGRAD_STREAM=$v', d['value'], d['ms_per_step'])"
  done
done
