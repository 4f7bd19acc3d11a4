# round-6 check: (optional) full GPU suite, smoke, the bench line with its traced roofline.
#   bash tools/gpu_r6.sh TAG [tests|notests] [extra bench args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r6}
MODE=${2:-tests}
shift 2 2>/dev/null
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
if [ "$MODE" = "tests" ]; then
  timeout -k 10 600 $PT tests -m gpu > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -2 gpurun_out/${TAG}_smoke.log
fi
timeout -k 10 900 python3 bench.py --trace-steps 10 --trace-out gpurun_out/${TAG}_kernel_stats.csv --shape-table gpurun_out/${TAG}_shape_table.txt "$@" > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench.log
python3 tools/step_profile.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_sorted.csv --steps 10 --bench gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_step_profile.txt || exit 1
cat gpurun_out/${TAG}_step_profile.txt
echo CHECK_DONE
