# whole-step A/B of the current build against build_ab/$1 (S2H_LIB_PATH), 2 rounds, 20 steps each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${1:-slp}
for r in 1 2; do
  for v in new $B; do
    if [ $v = new ]; then unset S2H_LIB_PATH; else export S2H_LIB_PATH=$PWD/build_ab/$v/libsam2hip.so; fi
    timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_ab_$v$r.log 2> gpurun_out/r4_ab_$v$r.err || { tail -5 gpurun_out/r4_ab_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_ab_$v$r.log'));print('$v', d['value'], d['ms_per_step'])"
  done
done
