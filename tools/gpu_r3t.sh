# kernel trace of the bench step (current build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3t_tr -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r3t_tr.log 2>&1 || exit 1
tail -1 $GRAFT_REPO_ROOT/gpurun_out/r3t_tr.log | cut -c1-120
