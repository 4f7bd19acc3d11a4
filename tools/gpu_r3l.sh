# dropout cost in the flash forward (attn_ab with and without dropout) + loss-kernel timing in a traced step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_ab.py --iters 10 --drop 0.1 > gpurun_out/r3l_d1.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/attn_ab.py --iters 10 --drop 0.0 > gpurun_out/r3l_d0.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r3l_d1.log gpurun_out/r3l_d0.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3l_tr -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline 0 --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r3l_tr.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/trace_diff.py gpurun_out/r3g_trB/tr_results.db $(find gpurun_out/r3l_tr -name "*.db" | head -1) --top 25
