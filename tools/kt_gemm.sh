# GPU kernel time (rocprofv3 kernel trace) of tools/gemm_one.py over a list of "M N K cfg" cases
# usage: bash tools/kt_gemm.sh "M N K cfg" ...     (cfg = tiling | dbg << 8, see s2h_gemm_config)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ktg
for c in "$@"; do
  tag=$(echo $c | tr ' ' _)
  set -- $c
  timeout -k 10 60 rocprofv3 --kernel-trace -d gpurun_out/ktg/$tag -o kt -- python3 tools/gemm_one.py $1 $2 $3 20 $4 > gpurun_out/ktg/$tag.log 2>&1 || { echo "FAILED $c"; exit 1; }
done
python3 - <<'PY'
import sqlite3, glob, os
for f in sorted(glob.glob("gpurun_out/ktg/*/kt_results.db"), key=os.path.getmtime):
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    d = [dict(zip(cols, r)) for r in c.execute("select * from kernels")]
    durs = sorted((x["end"] - x["start"]) / 1e3 for x in d if "gemm16" in str(x.get("name", "")))
    print(f"{f.split('/')[2]:28s} n={len(durs)} median {durs[len(durs) // 2]:8.1f} us  min {durs[0]:8.1f}")
PY
rm -rf gpurun_out/ktg
