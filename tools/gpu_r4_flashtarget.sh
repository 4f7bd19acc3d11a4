# round 4: flash forward key-split target (workgroups) in the step: S2H_ATTN_CFG = 1 | target << 8
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for t in 256 128 384 512; do
    v=$((1 + (t << 8)))
    S2H_ATTN_CFG=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_ft_$t$r.log 2> gpurun_out/r4_ft_$t$r.err || { tail -5 gpurun_out/r4_ft_$t$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_ft_$t$r.log'));print('flash target $t', d['value'], d['ms_per_step'])"
  done
done
