# round 4: config-5 MX-fp8 vs bf16 twin, then the profile (kernel trace of the timed replays + counter passes)
set -o pipefail
bash tools/gpu_r4_c5.sh r04_v8_c5 && NO_PMC= bash tools/gpu_prof4.sh r04_v8 10
