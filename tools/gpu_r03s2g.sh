#!/bin/bash
# 64 x 1080p under rocprofv3 kernel + memory-copy traces (the tracer serialises the
# lanes, so this gives each operation's own duration and count per frame)
set -e
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r03s2g
mkdir -p $O
cd /tmp && GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 > $R/$O/bench_prof.log 2>&1
