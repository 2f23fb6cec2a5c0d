#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/r02o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > $O/stream_tests.log 2>&1
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0"
timeout -k 10 200 $B > $O/bench_8k.log 2>&1
timeout -k 10 200 $B --config 1 > $O/cfg_4k.log 2>&1
timeout -k 10 200 $B --config 3 --steps 2 --warmup 1 > $O/cfg_batch_d1.0.log 2>&1
