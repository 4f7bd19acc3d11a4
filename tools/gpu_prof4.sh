# round-4 profile: rocprofv3 kernel trace + stats of ONLY the timed graph replays (between
# bench.py's trace markers), then separate counter passes (FETCH_SIZE, WRITE_SIZE, SQ set) over 2
# eager steps of tools/step_once.py for the GEMM / attention kernels.
#   bash tools/gpu_prof4.sh TAG [STEPS]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-prof}
STEPS=${2:-10}
RX='gemm|flash|attn_'
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_kt -o kt -- python3 bench.py --no-trace --steps $STEPS --warmup 3 --cpu-baseline 0 > gpurun_out/${TAG}_kt_bench.log 2>&1 || { echo KT_FAILED; tail -20 gpurun_out/${TAG}_kt_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_kt_bench.log | cut -c1-200
python3 tools/step_profile.py gpurun_out/${TAG}_kt gpurun_out/${TAG}_kernel_stats.csv --steps $STEPS --bench gpurun_out/${TAG}_kt_bench.log || exit 1
if [ -n "$NO_PMC" ]; then echo PROF_DONE; exit 0; fi
i=0
for set in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "$RX" -f csv -d gpurun_out/${TAG}_pmc$i -o pmc -- python3 tools/step_once.py 2 > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "PMC_PASS_${i}_FAILED"; tail -5 gpurun_out/${TAG}_pmc$i.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pmc$i.log
done
echo PROF_DONE
