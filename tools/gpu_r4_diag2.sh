set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/tape_diff.py --dtype bf16 --frames 8 --size 512 > gpurun_out/r4_tape_bf16.log 2>&1 || { tail -30 gpurun_out/r4_tape_bf16.log; exit 1; }
cat gpurun_out/r4_tape_bf16.log
