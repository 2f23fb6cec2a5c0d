#!/bin/bash
# same-box A/B of library builds through bench.py: bash tools/gpu_ab_bench.sh TAG "bench args" lib1 lib2 ...
set -e
export TMPDIR=/tmp
TAG=$1; shift
BARGS=$1; shift
R=$PWD
mkdir -p gpurun_out/$TAG
for round in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    JXG_LIB_PATH=$R/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 $BARGS > gpurun_out/$TAG/${n}_$round.log 2>&1
  done
done
