# in-call A/B of two library builds on the bench: A = build_ab/A/libsam2hip.so, B = this tree's
#   bash tools/ab_bench.sh [rounds]
set -o pipefail
R=${1:-2}
for i in $(seq 1 $R); do
  S2H_LIB_PATH=build_ab/A/libsam2hip.so timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 30 --warmup 5 > gpurun_out/abA_$i.log 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 30 --warmup 5 > gpurun_out/abB_$i.log 2>/dev/null || exit 1
  echo "A $(grep -o "\"value\": [0-9.]*" gpurun_out/abA_$i.log | head -1)  B $(grep -o "\"value\": [0-9.]*" gpurun_out/abB_$i.log | head -1)"
done
