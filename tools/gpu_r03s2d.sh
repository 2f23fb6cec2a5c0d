#!/bin/bash
# completion workers x lane batches: stream parity, 64 x 1080p sweep, 8K default bench
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_filters.py -x -v --timeout 200 --timeout-method thread > $O/gpu_stream.log 2>&1
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 6 --warmup 3"
for w in 0 1 2 3; do
  for k in 1 4; do
    JXG_PIPE_WORKERS=$w JXG_PIPE_BATCH=$k timeout -k 10 200 $B > $O/cfg3_w${w}_k$k.log 2>&1
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality > $O/bench_8k.log 2>&1
JXG_PIPE_WORKERS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/bench_8k_w0.log 2>&1
