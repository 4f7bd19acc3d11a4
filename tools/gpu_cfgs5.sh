# round-5: the other single-GPU BASELINE configurations, each bench line with the rocprofv3 trace of its
# own timed replays (bench.py --trace-out), then the stock-torch / small-kernel call sites of the bench step.
#   bash tools/gpu_cfgs5.sh TAG
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-cfg}
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --trace-steps 5 \
    --trace-out gpurun_out/${TAG}_${name}_kernel_stats.csv "$@" > gpurun_out/${TAG}_${name}.log 2> gpurun_out/${TAG}_${name}.err \
    || { echo "BENCH_${name}_FAILED"; tail -20 gpurun_out/${TAG}_${name}.err; return 1; }
  cut -c1-300 gpurun_out/${TAG}_${name}.log
}
run config3 --image-size 384 --frames 10 --objects 7 &&
run config4 --size large --image-size 1024 --frames 8 --objects 13 &&
run config5_fp8 --config 5 &&
run config5_bf16 --config 5 --dtype bf16 || exit 1
timeout -k 10 300 python3 tools/native_sites.py --top 40 > gpurun_out/${TAG}_native_sites.txt 2>&1 || { echo SITES_FAILED; tail -5 gpurun_out/${TAG}_native_sites.txt; exit 1; }
timeout -k 10 300 python3 tools/native_sites.py --top 120 --ops s2h_ln_wgrad_finalize,s2h_layernorm_bwd,s2h_colsum,s2h_window,s2h_add,s2h_add_bcast,s2h_sum_outer,s2h_layernorm_fwd > gpurun_out/${TAG}_ops_sites.txt 2>&1 || { echo OPS_SITES_FAILED; tail -5 gpurun_out/${TAG}_ops_sites.txt; exit 1; }
echo CFGS_DONE
