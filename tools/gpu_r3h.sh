# cold-cache GEMM tiling sweeps (forward / dgrad and weight gradients)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/gemm_cfg_sweep.py --cold > gpurun_out/r3h_cold_fwd.log 2>&1 || { tail gpurun_out/r3h_cold_fwd.log; exit 1; }
grep -v amdgpu gpurun_out/r3h_cold_fwd.log
timeout -k 10 500 python -u tools/gemm_cfg_sweep.py --cold --wgrad > gpurun_out/r3h_cold_wgrad.log 2>&1 || { tail gpurun_out/r3h_cold_wgrad.log; exit 1; }
grep -v amdgpu gpurun_out/r3h_cold_wgrad.log
