# round-6 in-call A/B of the whole bench step over the values of one environment switch (alternating
# order, two rounds), plus optional tool commands first.
#   bash tools/gpu_r6_ab.sh TAG VAR "v1 v2" ["tool command; ..."]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; VAR=$2; VALS=$3; PRE=$4
if [ -n "$PRE" ]; then
  timeout -k 10 300 bash -c "$PRE" > gpurun_out/${TAG}_pre.log 2>&1 || { echo PRE_FAILED; tail -30 gpurun_out/${TAG}_pre.log; exit 1; }
  cat gpurun_out/${TAG}_pre.log | grep -v amdgpu.ids
fi
for r in 1 2; do
  i=0
  for v in $VALS; do
    i=$((i+1))
    L=gpurun_out/${TAG}_ab_${i}_$r.log
    env $VAR=$v timeout -k 10 300 python3 bench.py --no-trace --no-prof --cpu-baseline 0 --steps 20 --warmup 3 > $L 2>&1 || { echo AB_FAILED; tail -20 $L; exit 1; }
    echo "$VAR=$v round $r: $(tail -1 $L | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
echo AB_DONE
