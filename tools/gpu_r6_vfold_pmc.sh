# PMC passes over the V-fold backward (tools/vfold_bwd_bench.py, one variant): stall split of the dK /
# dQ kernels.  bash tools/gpu_r6_vfold_pmc.sh TAG VARIANT
set -o pipefail
export TMPDIR=/tmp
TAG=$1; V=${2:-1}
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_avail.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "flash_bwd" -f csv -d gpurun_out/${TAG}_pmc$i -o pmc -- python3 tools/vfold_bwd_bench.py --variants $V --iters 2 --rounds 1 > gpurun_out/${TAG}_pmc$i.log 2>&1 || { echo "PMC_PASS_${i}_FAILED"; tail -5 gpurun_out/${TAG}_pmc$i.log; [ $i -eq 3 ] && exit 0; exit 1; }
  echo "pass $i ok"
done
