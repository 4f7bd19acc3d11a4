set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 0 1; do
  env S2H_FFN_FWD=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --no-trace --steps 20 --warmup 3 > gpurun_out/r05_v51_ffn$v.log 2> gpurun_out/r05_v51_ffn$v.err || { echo FAILED; tail -5 gpurun_out/r05_v51_ffn$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05_v51_ffn$v.log'));print('S2H_FFN_FWD=$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r05_v51_ffn_ab.txt
done
