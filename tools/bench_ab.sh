#!/bin/bash
# Headline-only bench (300 streamed 8K frames, cjxl preset) for the product
# library and variant builds (tools/ab/libjxg_NAME.so), twice each, same box.
# Usage: bash tools/bench_ab.sh TAG NAME...
set -e
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
  for n in base "$@"; do
    L=$PWD/jpeg-xl-lossy-image-compression-thesis_amd/jxg/libjxg.so
    [ $n != base ] && L=$PWD/tools/ab/libjxg_$n.so
    JXG_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --no-single --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 --alt-e4 0 > $O/b_${n}_${r}.log 2>&1
    echo "$n $(tail -1 $O/b_${n}_${r}.log | cut -c1-160)" >> $O/sum.txt
  done
done
