#!/bin/bash
# Experiment builds: tools/build_variant.sh NAME "EXTRA HIPCC FLAGS" -> tools/var/libjxg_NAME.so
# (bench.py / tests pick one up with JXG_LIB_PATH=...; the product is libjxg.so)
set -e
NAME=$1; FLAGS=$2
D=$(cd "$(dirname "$0")/.." && pwd)
P=$D/jpeg-xl-lossy-image-compression-thesis_amd
O=$D/tools/var/obj_$NAME
mkdir -p $O
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wno-unused-function $FLAGS"
pids=()
for f in $P/csrc/*.hip $(ls $P/csrc/*.cpp | grep -v jxg_cjxl); do
  b=$(basename $f); /opt/rocm/bin/hipcc $HIPFLAGS -c $f -o $O/${b%.*}.o 2>/dev/null & pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o $D/tools/var/libjxg_$NAME.so $O/*.o 2>/dev/null
rm -rf $O
echo built tools/var/libjxg_$NAME.so
