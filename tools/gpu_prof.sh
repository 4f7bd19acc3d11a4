# one GPU call: rocprofv3 kernel trace + stats of the bench, then FETCH_SIZE / WRITE_SIZE passes on the
# dominant attention-forward kernel (separate PMC passes, MI355X_MICROARCH.md "rocprofv3 PMC slots")
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-prof}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_kt -o kt -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/${TAG}_kt_bench.log 2>&1 || { echo KT_FAILED; tail -20 gpurun_out/${TAG}_kt_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_kt_bench.log
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex flash_fwd_kernel -f csv -d gpurun_out/${TAG}_fetch -o pmc -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --no-prof > gpurun_out/${TAG}_fetch.log 2>&1 || { echo FETCH_FAILED; tail -20 gpurun_out/${TAG}_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex flash_fwd_kernel -f csv -d gpurun_out/${TAG}_write -o pmc -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --no-prof > gpurun_out/${TAG}_write.log 2>&1 || { echo WRITE_FAILED; tail -20 gpurun_out/${TAG}_write.log; exit 1; }
find gpurun_out/${TAG}_* -name "*.csv" | head -20
