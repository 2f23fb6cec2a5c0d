#!/bin/bash
# merge kernels' occupancy vs spills: eval WPE 4 (8 spills) vs 3 (131 VGPRs, no spills),
# write WPE 3 (14 spills) vs 2 (199 VGPRs, no spills); 8K bench, two rounds interleaved
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2h
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0"
for r in 1 2; do
  timeout -k 10 200 $B > $O/prod_r$r.log 2>&1
  for v in eval3 write2 e3w2; do
    JXG_LIB_PATH=tools/var/libjxg_$v.so timeout -k 10 200 $B > $O/${v}_r$r.log 2>&1
  done
done
