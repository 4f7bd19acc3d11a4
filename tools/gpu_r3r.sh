# stock-kernel sites of the eager step (TorchDispatchMode)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/native_sites.py > gpurun_out/r3r_sites.log 2>&1 || { tail -30 gpurun_out/r3r_sites.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3r_sites.log | head -70
