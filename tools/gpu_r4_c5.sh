# config 5 (B+ 512^2, 16 frames, MX-fp8) vs its bf16 twin, and a kernel trace of the fp8 run
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r04_c5}
timeout -k 10 400 python -u bench.py --config 5 --cpu-baseline 0 --steps 10 --warmup 3 > gpurun_out/${T}_fp8.log 2> gpurun_out/${T}_fp8.err || { tail -5 gpurun_out/${T}_fp8.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_fp8.log'));print('fp8', d['value'], d['ms_per_step'], json.dumps(d['roofline']['families']))"
timeout -k 10 400 python -u bench.py --config 5 --dtype bf16 --cpu-baseline 0 --steps 10 --warmup 3 > gpurun_out/${T}_bf16.log 2> gpurun_out/${T}_bf16.err || { tail -5 gpurun_out/${T}_bf16.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${T}_bf16.log'));print('bf16', d['value'], d['ms_per_step'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --config 5 --steps 5 --warmup 2 --cpu-baseline 0 --no-prof > gpurun_out/${T}_kt_bench.log 2>&1 || { echo KT_FAILED; tail -20 gpurun_out/${T}_kt_bench.log; exit 1; }
python3 tools/step_profile.py gpurun_out/${T}_kt gpurun_out/${T}_kernel_stats.csv --steps 5
