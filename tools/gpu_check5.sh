# round-5 change check: targeted kernel tests, the parity / training-step suites, the bench line with
# its traced roofline, and an in-call A/B of one environment switch.
#   bash tools/gpu_check5.sh TAG "pytest -k expr" ENVVAR
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-chk}
KEXPR=${2:-window_pad}
ABVAR=${3:-}
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT tests/test_kernels_gpu.py -k "$KEXPR" > gpurun_out/${TAG}_ktest.log 2>&1 || { echo KTEST_FAILED; tail -30 gpurun_out/${TAG}_ktest.log; exit 1; }
tail -1 gpurun_out/${TAG}_ktest.log
timeout -k 10 600 $PT tests/test_parity_gpu.py tests/test_training_step_gpu.py > gpurun_out/${TAG}_parity.log 2>&1 || { echo PARITY_FAILED; tail -40 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
timeout -k 10 900 python3 bench.py --trace-steps 10 --trace-out gpurun_out/${TAG}_kernel_stats.csv > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench.log
python3 tools/step_profile.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_sorted.csv --steps 10 --bench gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_step_profile.txt || exit 1
cat gpurun_out/${TAG}_step_profile.txt
if [ -n "$ABVAR" ]; then
  for v in 0 1 0 1; do
    env $ABVAR=$v timeout -k 10 300 python3 bench.py --no-trace --no-prof --cpu-baseline 0 --steps 20 --warmup 3 > gpurun_out/${TAG}_ab_$v.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/${TAG}_ab_$v.log; exit 1; }
    echo "$ABVAR=$v $(tail -1 gpurun_out/${TAG}_ab_$v.log | cut -c1-120)"
  done
fi
echo CHECK_DONE
