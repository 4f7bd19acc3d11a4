# GPU kernel time by kernel name (rocprofv3 kernel trace) of one python command
# usage: bash tools/kt_run.sh TAG python3 tools/ln_one.py 13312 256
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/ktr
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/ktr/$tag -o kt -- "$@" > gpurun_out/ktr/$tag.log 2>&1 || { echo "FAILED $tag"; tail -5 gpurun_out/ktr/$tag.log; exit 1; }
python3 - "$tag" <<'PY'
import sqlite3, glob, sys, collections
for f in glob.glob(f"gpurun_out/ktr/{sys.argv[1]}/kt_results.db"):
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    by = collections.defaultdict(list)
    for r in c.execute("select * from kernels"):
        d = dict(zip(cols, r))
        by[str(d.get("name", ""))[:70]].append((d["end"] - d["start"]) / 1e3)
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"{sys.argv[1]:10s} {k:70s} n={len(v):4d} median {v[len(v) // 2]:8.1f} us")
PY
rm -rf gpurun_out/ktr/$tag
