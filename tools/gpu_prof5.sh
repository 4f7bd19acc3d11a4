# round-5 profile: bench.py with its own traced run (--trace-out: the per-kernel CSV of the traced
# timed replays that the bench line's roofline is computed from), the step profile from that same
# CSV and bench line, then separate counter passes (FETCH_SIZE, WRITE_SIZE, SQ set) over 2 eager
# steps of tools/step_once.py for the GEMM / attention kernels.
#   bash tools/gpu_prof5.sh TAG [STEPS] [extra bench args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-prof}
STEPS=${2:-10}
shift 2 2>/dev/null
RX='gemm|flash|attn_|ffn_'
timeout -k 10 900 python3 bench.py --trace-steps $STEPS --trace-out gpurun_out/${TAG}_kernel_stats.csv "$@" > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_bench.log
python3 tools/step_profile.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_sorted.csv --steps $STEPS --bench gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_step_profile.txt || exit 1
cat gpurun_out/${TAG}_step_profile.txt
if [ -n "$NO_PMC" ]; then echo PROF_DONE; exit 0; fi
i=0
for set in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "$RX" -f csv -d gpurun_out/${TAG}_pmc$i -o pmc -- python3 tools/step_once.py 2 > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "PMC_PASS_${i}_FAILED"; tail -5 gpurun_out/${TAG}_pmc$i.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pmc$i.log
done
echo PROF_DONE
