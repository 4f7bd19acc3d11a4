# counter passes over one GEMM shape (one rocprofv3 run per pass)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex gemm16 -f csv -d gpurun_out/pmc/p$i -o pmc -- python3 tools/gemm_one.py "$@" > gpurun_out/pmc/p$i.log 2>&1 || { echo PASS_$i_FAILED; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:28s} {sum(v)/len(v):16.1f}")
PY
