#!/bin/bash
# 64 x 1080p: product build vs a build without the per-frame timing markers
# (4 fewer commands per frame) -- is the small-frame stream bound by commands?
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2f
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 12 --warmup 3"
for r in 1 2; do
  JXG_PIPE_BATCH=1 timeout -k 10 200 $B > $O/prod_k1_r$r.log 2>&1
  JXG_LIB_PATH=tools/var/libjxg_lean.so JXG_PIPE_BATCH=1 timeout -k 10 200 $B > $O/lean_k1_r$r.log 2>&1
  JXG_PIPE_BATCH=4 timeout -k 10 200 $B > $O/prod_k4_r$r.log 2>&1
  JXG_LIB_PATH=tools/var/libjxg_lean.so JXG_PIPE_BATCH=4 timeout -k 10 200 $B > $O/lean_k4_r$r.log 2>&1
done
