#!/bin/bash
# streaming (pipelined) encode: GPU tests, default bench (ANS, pipelined), kernel stats
set -e
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-r02h}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 200 --timeout-method thread > $O/stream_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality > $O/bench.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 > $R/$O/bench_prof.log 2>&1
