# counter passes over the memory-attention flash kernels as the step runs them (tools/attn_ab.py:
# frame-table backward with keep bitmaps, forward with dropout) -- one rocprofv3 run per pass
#   bash tools/gpu_pmc_flash.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-flash}
mkdir -p gpurun_out/$TAG
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "flash_" -f csv -d gpurun_out/$TAG/p$i -o pmc -- python3 tools/attn_ab.py --iters 3 > gpurun_out/$TAG/p$i.log 2>&1 || { echo "PASS_${i}_FAILED"; tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
python3 - "$TAG" <<'PY'
import csv, glob, collections, sys
tag = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"gpurun_out/{tag}/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Grid_Size"])
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    print(k[0], "grid", k[1], "n", max(len(v) for v in cs.values()))
    for c, v in sorted(cs.items()):
        print(f"   {c:26s} {sum(v)/len(v):16.1f}")
PY
