#!/bin/bash
# Quick loop: GPU parity tests (optionally a -k filter), one bench line, kernel stats.
# Usage: bash tools/gpu_quick.sh TAG [pytest -k expr] 
set -e
export TMPDIR=/tmp
TAG=${1:-quick}; K=${2:-}
R=$PWD
mkdir -p gpurun_out/$TAG
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/$TAG/tests.log 2>&1
else
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
fi
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/$TAG/bench.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/$TAG/bench_prof.log 2>&1
