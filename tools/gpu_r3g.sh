# whole-step A/B with kernel traces of both builds (A = build_ab/A) and the per-kernel difference
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_bench.sh 1 || exit 1
cd /tmp
S2H_LIB_PATH=$GRAFT_REPO_ROOT/build_ab/A/libsam2hip.so timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3g_trA -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r3g_trA.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3g_trB -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r3g_trB.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 tools/trace_diff.py $(find gpurun_out/r3g_trA -name "*.db" | head -1) $(find gpurun_out/r3g_trB -name "*.db" | head -1) --top 30
