#!/bin/bash
# 64 x 1080p host profile of the submitting thread, K = 1 / 4 (JXG_PIPE_PROFILE build)
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2c
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 6 --warmup 3"
for k in 1 4; do
  JXG_LIB_PATH=tools/var/libjxg_pprof.so JXG_PIPE_BATCH=$k timeout -k 10 200 $B > $O/cfg3_pprof_k$k.log 2>&1
done
