#!/bin/bash
# 64 x 1080p: fewer physical lanes (hardware queues) x more batch slots
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2i
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 8 --warmup 3"
for lk in "12 1" "4 8" "6 6" "8 4" "3 8" "2 8"; do
  set -- $lk
  JXG_PIPE_MAX_LANES=$1 JXG_PIPE_BATCH=$2 timeout -k 10 200 $B > $O/cfg3_l$1_k$2.log 2>&1
done
