# 16-B AdamW form: its bit-identity test + the optimizer / step tests, then an in-call A/B of the whole
# step against the previous optim.hip (build_ab/adam_old, S2H_LIB_PATH)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "adamw" tests/test_training_step_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_v24_adamw_tests.log 2>&1 || { tail -30 gpurun_out/r04_v24_adamw_tests.log; exit 1; }
tail -2 gpurun_out/r04_v24_adamw_tests.log
NEW=sam2-video-training_amd/sam2_video/_lib/libsam2hip.so
OLD=build_ab/adam_old/libsam2hip.so
for tag in old new old new; do
  if [ $tag = old ]; then L=$OLD; else L=$NEW; fi
  S2H_LIB_PATH=$L timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 30 > gpurun_out/ab_$tag.log 2> gpurun_out/ab_$tag.err || { echo "BENCH_FAILED $tag"; tail -20 gpurun_out/ab_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$tag.log'));print('$tag', d['value'], d['ms_per_step'])"
done 2>&1 | tee gpurun_out/r04_v24_adamw_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04_v24_kt -o kt -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --no-prof > gpurun_out/r04_v24_kt.log 2>&1 || { echo KT_FAILED; exit 1; }
grep -h adamw gpurun_out/r04_v24_kt/*kernel_stats.csv gpurun_out/r04_v24_kt/*/*kernel_stats.csv 2>/dev/null || true
