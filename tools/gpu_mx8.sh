# MX-fp8 kernels: layout probe + parity tests (run via gpurun from the repo root)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/probe_mx.hip -o /tmp/probe_mx 2>/dev/null
timeout -k 5 60 /tmp/probe_mx > gpurun_out/probe_mx.log 2>&1; echo "probe rc=$?"; grep -v "^  lane" gpurun_out/probe_mx.log
timeout -k 10 300 python -u -m pytest tests/test_mx8_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/mx8_tests.log 2>&1
rc=$?
tail -30 gpurun_out/mx8_tests.log
exit $rc
