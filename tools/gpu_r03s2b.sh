#!/bin/bash
# lane batches: stream parity (incl. K = 1/2/3/8), then 64 x 1080p ANS per K
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 200 --timeout-method thread > $O/gpu_stream.log 2>&1
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 6 --warmup 3"
for k in 1 2 3 4 8; do
  JXG_PIPE_BATCH=$k timeout -k 10 200 $B > $O/cfg3_k$k.log 2>&1
done
