# round-4 final check of the shipped build: full GPU suite, smoke, bench, then the profile (kernel trace
# of the timed replays + counter passes)
set -o pipefail
T=${1:-r04_final}
bash tools/gpu_r4_full.sh $T
rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_prof4.sh ${T}p 10
