# MX-fp8 model-level tests + config-5 bench (run via gpurun from the repo root)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_mx8_gpu.py tests/test_fp8_gpu.py -x -q -s -rf --timeout 240 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
rc=$?
grep -E "fp8 vs bf16|MX-fp8 GEMM|config 5 losses|passed|failed|Error" gpurun_out/fp8_tests.log | tail -20
[ $rc -eq 0 ] || { tail -40 gpurun_out/fp8_tests.log; exit $rc; }
timeout -k 10 400 python -u bench.py --config 5 --steps 10 --warmup 3 --cpu-baseline 0 --kernel-table > gpurun_out/bench_c5.log 2> gpurun_out/bench_c5.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.log
timeout -k 10 400 python -u bench.py --frames 16 --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_c5_bf16.log 2> gpurun_out/bench_c5_bf16.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_c5_bf16.err; exit 1; }
cat gpurun_out/bench_c5_bf16.log
