# round-6 sweep: the whole bench step for each value of one environment switch (one run each, the
# baseline value repeated between groups), printing value and ms/step.
#   bash tools/gpu_r6_sweep.sh TAG VAR "v1 v2 ..." [BASE]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; VAR=$2; VALS=$3; BASE=$4
i=0
for v in $VALS; do
  i=$((i+1))
  env $VAR="$v" timeout -k 10 300 python3 bench.py --no-trace --no-prof --cpu-baseline 0 --steps 20 --warmup 3 > gpurun_out/${TAG}_sw_$i.log 2>&1 || { echo "RUN_FAILED $v"; tail -20 gpurun_out/${TAG}_sw_$i.log; exit 1; }
  echo "$VAR=$v: $(tail -1 gpurun_out/${TAG}_sw_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo SWEEP_DONE
