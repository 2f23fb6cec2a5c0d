#!/bin/bash
# front-kernel A/B: GPU parity tests on the product, then one-at-a-time benches per lib
set -e
export TMPDIR=/tmp
TAG=$1; shift
R=$PWD
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
for round in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    JXG_LIB_PATH=$R/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --steps 20 > gpurun_out/$TAG/${n}_$round.log 2>&1
  done
done
