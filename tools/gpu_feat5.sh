# one GPU call for a step-level change: its tests + the step suites, the traced bench line and step
# profile, then an in-call A/B of its environment switch (VAR=A vs VAR=B, alternating, 20 steps each).
#   VAR=S2H_GRAD_DEFER A=0 B=1 bash tools/gpu_feat5.sh TAG "tests/test_x_gpu.py ..."
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-feat}
TESTS=${2:-}
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $PT $TESTS tests/test_determinism_gpu.py tests/test_graph_gpu.py tests/test_parity_gpu.py \
  tests/test_training_step_gpu.py tests/test_ddp_gpu.py > gpurun_out/${TAG}_suites.log 2>&1 || { echo SUITES_FAILED; tail -40 gpurun_out/${TAG}_suites.log; exit 1; }
tail -1 gpurun_out/${TAG}_suites.log
timeout -k 10 900 python3 bench.py --trace-steps 10 --trace-out gpurun_out/${TAG}_kernel_stats.csv > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-200 gpurun_out/${TAG}_bench.log
python3 tools/step_profile.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_sorted.csv --steps 10 --bench gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_step_profile.txt || exit 1
head -14 gpurun_out/${TAG}_step_profile.txt
ab() {  # VAR A B: alternating A/B of one switch
  local var=$1 a=$2 b=$3
  for v in "$a" "$b" "$a" "$b"; do
    env "$var=$v" timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --no-trace --steps 20 --warmup 3 > gpurun_out/${TAG}_ab_$var$v.log 2> gpurun_out/${TAG}_ab_$var$v.err || { echo "AB_FAILED $var=$v"; tail -20 gpurun_out/${TAG}_ab_$var$v.err; return 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_ab_$var$v.log'));print('$var=$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}_ab.txt
  done
}
if [ -n "$VAR" ]; then ab "$VAR" "$A" "$B" || exit 1; fi
if [ -n "$VAR2" ]; then ab "$VAR2" "$A" "$B" || exit 1; fi
echo CHECK_DONE
