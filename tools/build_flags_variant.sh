# build libsam2hip.so of this tree with extra device-compiler flags into build_ab/NAME/libsam2hip.so
# (A/B of code-generation options, selected at run time by S2H_LIB_PATH)
#   bash tools/build_flags_variant.sh NAME "<extra hipcc flags>"
set -e
NAME=$1; EXTRA=$2
D=build_ab/$NAME
rm -rf $D && mkdir -p $D/csrc $D/sam2_video/_lib
cp sam2-video-training_amd/csrc/* $D/csrc/ 2>/dev/null || true
rm -rf $D/csrc/build
make -C $D/csrc -j8 CXXFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $EXTRA" > $D/build.log 2>&1
cp $D/sam2_video/_lib/libsam2hip.so $D/libsam2hip.so && rm -rf $D/csrc $D/sam2_video
echo built $D/libsam2hip.so
