# round 4: in-call A/B of the default bench step, round-4 checkpoint build (37d4210, git worktree under
# build_ab/r4v1, its own libsam2hip.so) against HEAD
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  (cd build_ab/r4v1 && timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > ../../gpurun_out/r4_regr_old$r.log 2> ../../gpurun_out/r4_regr_old$r.err) || { tail -5 gpurun_out/r4_regr_old$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4_regr_old$r.log'));print('37d4210', d['value'], d['ms_per_step'])"
  timeout -k 10 300 python -u bench.py --cpu-baseline 0 --no-prof --steps 20 > gpurun_out/r4_regr_new$r.log 2> gpurun_out/r4_regr_new$r.err || { tail -5 gpurun_out/r4_regr_new$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4_regr_new$r.log'));print('HEAD', d['value'], d['ms_per_step'])"
done
