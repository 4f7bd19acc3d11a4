# Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only, this container):
# builds the prompt stage (csrc/prompts_host.cpp: opening, run-length 8-connected labelling,
# moments, one thread per category) as a host-only shared library with -fsanitize=address,undefined
# and runs its tests against it (S2H_HOST_LIB_PATH; libasan preloaded into python, any existing
# LD_PRELOAD kept after it).  Any ASan / UBSan report fails the run (halt_on_error).
#   bash tools/sanitize_host.sh
set -e -o pipefail
cd "$(dirname "$0")/.."
OUT=build_san
mkdir -p $OUT
g++ -O1 -g -std=c++17 -fPIC -shared -pthread -fno-omit-frame-pointer -fsanitize=address,undefined \
    -fno-sanitize-recover=all sam2-video-training_amd/csrc/prompts_host.cpp -o $OUT/libprompts_san.so
ASAN_LIB=$(g++ -print-file-name=libasan.so)
UBSAN_LIB=$(g++ -print-file-name=libubsan.so)
export S2H_HOST_LIB_PATH=$PWD/$OUT/libprompts_san.so
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
LD_PRELOAD="$ASAN_LIB:$UBSAN_LIB${LD_PRELOAD:+:$LD_PRELOAD}" python -m pytest -q -p no:cacheprovider \
    tests/test_prompts_native.py "tests/test_host.py::test_objects_and_prompts_match_reference" \
    tests/test_host.py::test_sanitizer_build_is_in_use 2>&1 | tee $OUT/sanitize.log
