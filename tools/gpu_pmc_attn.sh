# counter passes over tools/attn_one.py for one kernel regex (one rocprofv3 run per pass)
# usage: bash tools/gpu_pmc_attn.sh TAG REGEX "B H Lq Lk D iters p" "SET1" "SET2" ...
set -o pipefail
export TMPDIR=/tmp
tag=$1; rx=$2; args=$3; shift 3
mkdir -p gpurun_out/pmc_$tag
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "$rx" -f csv -d gpurun_out/pmc_$tag/p$i -o pmc -- python3 tools/attn_one.py $args > gpurun_out/pmc_$tag/p$i.log 2>&1 || { echo "PASS_${i}_FAILED"; tail -5 gpurun_out/pmc_$tag/p$i.log; exit 1; }
done
python3 - "$tag" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/pmc_{sys.argv[1]}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1])
for k, v in agg.items():
    print(f"  {k:28s} {sum(v)/len(v):16.1f}")
PY
