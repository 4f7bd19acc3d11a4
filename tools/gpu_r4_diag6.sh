# round 4: determinism of the step after -fno-slp-vectorize, and its cost (A/B against the SLP build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_determinism_gpu.py tests/test_vfold_gpu.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r4_det_tests.log 2>&1 || { tail -30 gpurun_out/r4_det_tests.log; exit 1; }
grep -i "passed\\|failed\\|fused vs" gpurun_out/r4_det_tests.log
timeout -k 10 400 python -u tools/tape_diff.py --dtype bf16 --frames 8 --size 512 --show 6 > gpurun_out/r4_tape3.log 2>&1 || { tail -30 gpurun_out/r4_tape3.log; exit 1; }
grep -v "      at" gpurun_out/r4_tape3.log | tail -30
timeout -k 10 400 python -u tools/replay_diff.py --dtype fp8 --frames 16 --size 512 > gpurun_out/r4_replay_fp8.log 2>&1 || { tail -30 gpurun_out/r4_replay_fp8.log; exit 1; }
grep "==\|first" gpurun_out/r4_replay_fp8.log
timeout -k 10 400 python -u tools/replay_diff.py --dtype bf16 --frames 8 --size 512 > gpurun_out/r4_replay_bf16.log 2>&1 || { tail -30 gpurun_out/r4_replay_bf16.log; exit 1; }
grep "==\|first" gpurun_out/r4_replay_bf16.log
for r in 1 2; do
  for v in new slp; do
    if [ $v = new ]; then unset S2H_LIB_PATH; else export S2H_LIB_PATH=$PWD/build_ab/$v/libsam2hip.so; fi
    timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_ab_$v$r.log 2> gpurun_out/r4_ab_$v$r.err || { tail -5 gpurun_out/r4_ab_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_ab_$v$r.log'));print('$v', d['value'], d['ms_per_step'])"
  done
done
