set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default noslp precise; do
  if [ $v = default ]; then unset S2H_LIB_PATH; else export S2H_LIB_PATH=$PWD/build_ab/$v/libsam2hip.so; fi
  echo "== library $v"
  timeout -k 10 300 python -u tools/determinism_probe.py --gemm-variants --reps 30 > gpurun_out/r4_detprobe_$v.log 2>&1 || { tail -30 gpurun_out/r4_detprobe_$v.log; exit 1; }
  grep -v "rep " gpurun_out/r4_detprobe_$v.log
done
