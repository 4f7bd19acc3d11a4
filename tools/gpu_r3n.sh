# tiny-M GEMM tilings inside the step: env A/B over S2H_GEMM_TINY_CFG (0 auto, 18 = 64^2 4-stage, 19 = 64^2 32-deep 8-stage)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 19 18 0 19 18; do
  S2H_GEMM_TINY_CFG=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/tiny_$v.log 2> gpurun_out/tiny_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tiny_$v.log'));print('TINY=$v', d['value'], d['ms_per_step'])"
done
