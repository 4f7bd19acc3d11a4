set -o pipefail
export TMPDIR=/tmp
for c in 1 7 2; do
S2H_GEMM_CFG=$c timeout -k 10 300 python -u bench.py --kernel-table > gpurun_out/bench_c$c.log 2> gpurun_out/bench_c$c.err || exit 1
done
