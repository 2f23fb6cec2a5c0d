#!/bin/bash
# Iteration loop on the GPU box: GPU parity tests, one bench line, rocprof
# kernel summary.  Usage: bash tools/gpu_iter.sh TAG [bench args...]
set -e
export TMPDIR=/tmp
TAG=${1:-iter}; shift || true
R=$PWD
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/$TAG/bench.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $R/gpurun_out/$TAG/bench_prof.log 2>&1
