# one GPU call: rocprofv3 kernel trace + stats of the bench, then separate counter passes
# (MI355X_MICROARCH.md rocprofv3 PMC limits: FETCH_SIZE and WRITE_SIZE each in its own pass, <= 8
# SQ counters) over 2 eager steps of tools/step_once.py for the GEMM / attention kernels.
#   bash tools/gpu_prof2.sh TAG
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-prof}
RX='gemm|flash|attn_'
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_kt -o kt -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/${TAG}_kt_bench.log 2>&1 || { echo KT_FAILED; tail -20 gpurun_out/${TAG}_kt_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_kt_bench.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
i=0
for set in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "$RX" -f csv -d gpurun_out/${TAG}_pmc$i -o pmc -- python3 tools/step_once.py 2 > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "PMC_PASS_${i}_FAILED"; tail -5 gpurun_out/${TAG}_pmc$i.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pmc$i.log
done
echo PROF_DONE
