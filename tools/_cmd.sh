set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash or attention or attn" -x -q --timeout 120 --timeout-method thread > gpurun_out/fl.log 2>&1 || { tail -30 gpurun_out/fl.log; exit 1; }
tail -2 gpurun_out/fl.log
timeout -k 10 200 python -u tools/attn_bench.py --iters 20 > gpurun_out/attn.log 2>&1 || exit 1
cat gpurun_out/attn.log
[ -n "$NOBENCH" ] || timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || exit 1
[ -n "$NOBENCH" ] || cat gpurun_out/bench.log
