# round-3 checkpoint: every GPU test, smoke, bench (CPU baseline included), then kernel stats + PMC passes
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round.sh || exit 1
bash tools/gpu_prof2.sh ${TAG:-r03_v12} || exit 1
