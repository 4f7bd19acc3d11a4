# informational: the bench step with dropout off (bench.py --dropout 0) under the kernel trace, to price
# the dropout work inside the attention / GEMM kernels against the default trace of the same call
#   bash tools/gpu_drop0.sh TAG
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-drop0}
timeout -k 10 600 python3 bench.py --dropout 0 --cpu-baseline 0 --trace-steps 10 --trace-out gpurun_out/${TAG}_kernel_stats.csv > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-200 gpurun_out/${TAG}_bench.log
python3 tools/step_profile.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_sorted.csv --steps 10 --bench gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_step_profile.txt || exit 1
head -12 gpurun_out/${TAG}_step_profile.txt
