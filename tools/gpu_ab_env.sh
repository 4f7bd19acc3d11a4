# A/B of one environment switch inside ONE GPU call (same box): the default bench with VAR=a, VAR=b,
# VAR=a, VAR=b (20 timed steps each, no profiling).   VAR=S2H_VFOLD A=0 B=1 bash tools/gpu_ab_env.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$A" "$B" "$A" "$B"; do
  env "$VAR=$v" timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps ${STEPS:-20} ${BENCH_ARGS} > gpurun_out/ab_$v.log 2> gpurun_out/ab_$v.err || { echo "BENCH_FAILED $VAR=$v"; tail -20 gpurun_out/ab_$v.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/ab_$v.log'));print('$VAR=$v', d['value'], d['ms_per_step'])"
done
