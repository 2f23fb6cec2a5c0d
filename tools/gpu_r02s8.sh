#!/bin/bash
# 8K pipeline depth after the merge_eval speed-up: 6 / 7 (default) / 8 lanes,
# default bench without side legs, two rounds on one box
set -e
export TMPDIR=/tmp
O=gpurun_out/r02s8
R=$PWD
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0"
for r in 1 2; do
  for n in ch64 d6 d8; do
    JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 200 $B > $O/b8k_${n}_$r.log 2>&1
  done
done
