#!/bin/bash
# same-box A/B at 100 timed frames, three rounds: bash tools/gpu_ab100.sh TAG lib1 lib2 ...
set -e
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for round in 1 2 3; do
  for L in "$@"; do
    n=$(basename $L .so)
    JXG_LIB_PATH=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --steps 100 $BENCH_EXTRA > gpurun_out/$TAG/${n}_$round.log 2>&1
  done
done
