# in-call A/B of the flash forward's key-split target (S2H_ATTN_CFG = 1 | target << 8; 256 = default)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-attn_target}
for cfg in 65537 32769 131073 65537 32769 131073; do
  env S2H_ATTN_CFG=$cfg timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --no-trace --steps 20 --warmup 3 > gpurun_out/${TAG}_$cfg.log 2> gpurun_out/${TAG}_$cfg.err || { echo "FAILED $cfg"; tail -20 gpurun_out/${TAG}_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$cfg.log'));print('S2H_ATTN_CFG=$cfg target', $cfg >> 8, d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}.txt
done
