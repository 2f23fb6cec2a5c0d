#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --alt-ans-streams 0 --alt-thesis 0 --no-quality > $O/bench_cfg3.log 2>&1
