# round 4: split-K workgroup target with the split-major order -- bench step per S2H_GEMM_SPLIT_TARGET
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in 768 512 1024 1536; do
    S2H_GEMM_SPLIT_TARGET=$v timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_st_$v$r.log 2> gpurun_out/r4_st_$v$r.err || { tail -5 gpurun_out/r4_st_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_st_$v$r.log'));print('S2H_GEMM_SPLIT_TARGET=$v', d['value'], d['ms_per_step'])"
  done
done
