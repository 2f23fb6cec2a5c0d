#!/bin/bash
# full GPU tests + default bench + kernel stats: bash tools/gpu_full.sh TAG
set -e
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
cd /tmp && GPU_MAX_HW_QUEUES=16 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 > $R/$O/bench_prof.log 2>&1
