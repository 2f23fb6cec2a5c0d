#!/bin/bash
set -e
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r02q
mkdir -p $O
cd /tmp && GPU_MAX_HW_QUEUES=16 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 1 --warmup 1 > $R/$O/bench_prof.log 2>&1
