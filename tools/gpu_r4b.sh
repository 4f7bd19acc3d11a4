# V-fold dK store with the inverse RoPE fused: kernel / V-fold / frame-tape / step / parity tests, env A/B (S2H_VFOLD_DK_ROPE), trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_vfold_gpu.py tests/test_frametape_gpu.py tests/test_training_step_gpu.py tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -2 gpurun_out/r4b_tests.log
for v in 1 0 1; do
  S2H_VFOLD_DK_ROPE=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/v_win_$v.log 2> gpurun_out/v_win_$v.err || { tail -5 gpurun_out/v_win_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/v_win_$v.log'));print('DKROPE=$v', d['value'], d['ms_per_step'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r4b_tr -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r4b_tr.log 2>&1 || exit 1
tail -1 $GRAFT_REPO_ROOT/gpurun_out/r4b_tr.log | cut -c1-120
