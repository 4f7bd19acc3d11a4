# build libsam2hip.so from the csrc of git revision REV (with this tree's other sources) into
# abvar/NAME/libsam2hip.so (ABDIR overrides; abvar/ travels to the GPU box, build_ab/ does not) -- the A side of an in-call A/B (S2H_LIB_PATH)
#   bash tools/build_variant.sh NAME REV [files...]   (files: csrc sources taken from REV; default all)
set -e
NAME=$1; REV=$2; shift 2
D=${ABDIR:-abvar}/$NAME
rm -rf $D && mkdir -p $D/csrc $D/sam2_video/_lib
cp sam2-video-training_amd/csrc/* $D/csrc/ 2>/dev/null || true
if [ $# -eq 0 ]; then set -- $(git ls-tree --name-only $REV sam2-video-training_amd/csrc/ | xargs -n1 basename); fi
for f in "$@"; do git show $REV:sam2-video-training_amd/csrc/$f > $D/csrc/$f; done
rm -rf $D/csrc/build
make -C $D/csrc -j8 > $D/build.log 2>&1
cp $D/sam2_video/_lib/libsam2hip.so $D/libsam2hip.so && rm -rf $D/csrc $D/sam2_video
echo built $D/libsam2hip.so
