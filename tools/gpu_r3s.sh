# small-window attention kernels: attention tests, then in-step env A/B (S2H_ATTN_WIN 1 / 0)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "small_window or attention_fwd_bwd" > gpurun_out/r3s_tests.log 2>&1 || { tail -40 gpurun_out/r3s_tests.log; exit 1; }
tail -2 gpurun_out/r3s_tests.log
for v in 1 0 1 0; do
  S2H_ATTN_WIN=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/win_$v.log 2> gpurun_out/win_$v.err || { tail -5 gpurun_out/win_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/win_$v.log'));print('WIN=$v', d['value'], d['ms_per_step'])"
done
