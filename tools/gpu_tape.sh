# frame-tape bring-up: tape vs per-frame tests first, then the parity suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frametape_gpu.py -x -v -s --timeout 150 --timeout-method thread > gpurun_out/tape_tests.log 2>&1
rc=$?
tail -40 gpurun_out/tape_tests.log
if [ $rc -ne 0 ]; then echo "TAPE_TESTS rc=$rc"; exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
exit $rc
