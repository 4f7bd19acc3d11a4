set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/determinism_probe.py --gemm-variants --reps 30 > gpurun_out/r4_detprobe2.log 2>&1 || { tail -30 gpurun_out/r4_detprobe2.log; exit 1; }
grep -v "rep " gpurun_out/r4_detprobe2.log
