#!/bin/bash
set -e
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/ansprof
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ansprof/bench_default.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ansprof/prof -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --coder ans > $R/gpurun_out/ansprof/bench_prof.log 2>&1
