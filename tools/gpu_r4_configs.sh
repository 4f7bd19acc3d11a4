# the other single-GPU BASELINE configurations on the shipped build: config 3 (B+ 384^2, 10 frames,
# 7 objects) and config 4 (Hiera-L 1024^2, 8 frames, 13 objects)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --image-size 384 --frames 10 --objects 7 --cpu-baseline 0 --steps 10 --warmup 3 > gpurun_out/r04_v26_bench_config3_1gpu.log 2> gpurun_out/r04_v26_c3.err || { tail -20 gpurun_out/r04_v26_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04_v26_bench_config3_1gpu.log'));print('config3', d['value'], d['ms_per_step'], json.dumps(d['roofline']['families']))"
timeout -k 10 600 python -u bench.py --size large --image-size 1024 --frames 8 --objects 13 --cpu-baseline 0 --steps 10 --warmup 3 > gpurun_out/r04_v26_bench_config4_1gpu.log 2> gpurun_out/r04_v26_c4.err || { tail -20 gpurun_out/r04_v26_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04_v26_bench_config4_1gpu.log'));print('config4', d['value'], d['ms_per_step'], json.dumps(d['roofline']['families']))"
