# round 4: rocprofv3 kernel stats of the default bench (10 timed steps), round-4 checkpoint build
# (build_ab/r4v1) and HEAD, for a per-kernel diff of the two
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
(cd build_ab/r4v1 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../../gpurun_out/r4_kt_old -o kt -f csv -- python3 bench.py --cpu-baseline 0 --no-prof --steps 10 > ../../gpurun_out/r4_kt_old.log 2>&1) || { tail -5 gpurun_out/r4_kt_old.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_kt_new -o kt -f csv -- python3 bench.py --cpu-baseline 0 --no-prof --steps 10 > gpurun_out/r4_kt_new.log 2>&1 || { tail -5 gpurun_out/r4_kt_new.log; exit 1; }
grep -h '^{' gpurun_out/r4_kt_old.log gpurun_out/r4_kt_new.log | python3 -c "import sys,json;[print(json.loads(l)['ms_per_step']) for l in sys.stdin]"
