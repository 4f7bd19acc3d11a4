# stock-kernel sites of the eager step; in-step env A/B of the 4x1 wave-grid GEMMs (S2H_GEMM_W41 0 / 1 / 2)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/native_sites.py > gpurun_out/r3q_sites.log 2>&1 || { tail -30 gpurun_out/r3q_sites.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3q_sites.log | head -45
for v in 0 1 2 0 1 2; do
  S2H_GEMM_W41=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/w41_$v.log 2> gpurun_out/w41_$v.err || { tail -5 gpurun_out/w41_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/w41_$v.log'));print('W41=$v', d['value'], d['ms_per_step'])"
done
