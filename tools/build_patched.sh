#!/bin/bash
# Experiment builds from a patched copy of csrc/ (timing attribution only; the
# output is not expected to be bit-exact): tools/build_patched.sh NAME 'sed script' [FILE ...]
# -> tools/var/libjxg_NAME.so
set -e
NAME=$1; SED=$2; shift 2; FILES=${@:-jxg_front.hip}
D=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/jxgpatch.XXXX)
mkdir -p $T/p
cp -r $D/jpeg-xl-lossy-image-compression-thesis_amd/csrc $T/p/
cp -r $D/include $T/
for FILE in $FILES; do
  sed -i "$SED" $T/p/csrc/$FILE
  cmp -s $T/p/csrc/$FILE $D/jpeg-xl-lossy-image-compression-thesis_amd/csrc/$FILE && { echo "patch changed nothing in $FILE"; exit 1; }
done
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wno-unused-function"
pids=()
for f in $T/p/csrc/*.hip $(ls $T/p/csrc/*.cpp | grep -v jxg_cjxl); do
  b=$(basename $f); /opt/rocm/bin/hipcc $HIPFLAGS -c $f -o $T/${b%.*}.o & pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
mkdir -p $D/tools/var
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o $D/tools/var/libjxg_$NAME.so $T/*.o
rm -rf $T
echo built tools/var/libjxg_$NAME.so
