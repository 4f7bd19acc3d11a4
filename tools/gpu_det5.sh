# deterministic-finalize check: targeted kernel tests, determinism / graph / training-step / parity
# suites, the traced bench line and an optional env A/B (gpu_check5.sh without the parity step repeated)
#   bash tools/gpu_det5.sh TAG "pytest -k expr"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-det}
KEXPR=${2:-layernorm}
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 400 $PT tests/test_kernels_gpu.py -k "$KEXPR" > gpurun_out/${TAG}_ktest.log 2>&1 || { echo KTEST_FAILED; tail -30 gpurun_out/${TAG}_ktest.log; exit 1; }
tail -1 gpurun_out/${TAG}_ktest.log
timeout -k 10 700 $PT tests/test_determinism_gpu.py tests/test_graph_gpu.py tests/test_parity_gpu.py tests/test_training_step_gpu.py > gpurun_out/${TAG}_suites.log 2>&1 || { echo SUITES_FAILED; tail -40 gpurun_out/${TAG}_suites.log; exit 1; }
tail -1 gpurun_out/${TAG}_suites.log
timeout -k 10 900 python3 bench.py --trace-steps 10 --trace-out gpurun_out/${TAG}_kernel_stats.csv > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-200 gpurun_out/${TAG}_bench.log
python3 tools/step_profile.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_sorted.csv --steps 10 --bench gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_step_profile.txt || exit 1
head -14 gpurun_out/${TAG}_step_profile.txt
echo CHECK_DONE
