set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/determinism_probe.py --reps 20 > gpurun_out/r4_detprobe.log 2>&1 || { tail -30 gpurun_out/r4_detprobe.log; exit 1; }
cat gpurun_out/r4_detprobe.log
timeout -k 10 400 python -u tools/tape_diff.py --dtype bf16 --frames 4 --size 512 --show 6 > gpurun_out/r4_tape2.log 2>&1 || { tail -30 gpurun_out/r4_tape2.log; exit 1; }
cat gpurun_out/r4_tape2.log
