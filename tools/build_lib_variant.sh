#!/bin/bash
# Build libjxg.so from csrc/ of a git ref (or the working tree: "."), with
# optional replacement source files, into tools/ab/libjxg_NAME.so (same-box
# A/B runs select it with JXG_LIB_PATH; bit-exactness is checked on the box):
#   tools/build_lib_variant.sh NAME REF [csrc-file=path ...]
set -e
NAME=$1; REF=$2; shift 2
D=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/jxgvar.XXXX)
if [ "$REF" = "." ]; then
  cp -r $D/jpeg-xl-lossy-image-compression-thesis_amd/csrc $T/csrc
  cp -r $D/include $T/include
else
  mkdir -p $T/csrc $T/include
  git -C $D archive $REF jpeg-xl-lossy-image-compression-thesis_amd/csrc include | tar -x -C $T
  mv $T/jpeg-xl-lossy-image-compression-thesis_amd/csrc/* $T/csrc/; mv $T/include/* $T/include/ 2>/dev/null || true
fi
for kv in "$@"; do cp ${kv#*=} $T/csrc/${kv%%=*}; done
mkdir -p $T/x && ln -s $T/csrc $T/x/csrc && ln -s $T/include $T/include_ && true
# the sources include "../../include/jxg.h": lay them out as in the repo
mkdir -p $T/r/pkg && mv $T/csrc $T/r/pkg/csrc && mv $T/include $T/r/include
HF="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wno-unused-function"
pids=()
for f in $T/r/pkg/csrc/*.hip $(ls $T/r/pkg/csrc/*.cpp | grep -v jxg_cjxl); do
  b=$(basename $f); /opt/rocm/bin/hipcc $HF -c $f -o $T/${b%.*}.o & pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
mkdir -p $D/tools/ab
/opt/rocm/bin/hipcc $HF -shared -o $D/tools/ab/libjxg_$NAME.so $T/*.o
rm -rf $T
echo built tools/ab/libjxg_$NAME.so
